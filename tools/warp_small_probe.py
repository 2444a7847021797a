"""Device time of the warp backward at the decoder's level 1 (16x128x8x26) for the default
(binned gather) and variant 7 (small-image kernel), per need_x / need_flow, on zero and
2-px sinusoid flows (graph-replayed launches). GPU box: python tools/warp_small_probe.py"""
import sys, os, json
sys.path.insert(0, os.getcwd())
import torch
from unsamflow_amd import ops, _lib
from unsamflow_amd.kernel_timer import device_time_us, site_launcher
dev = torch.device("cuda:0")
lib = _lib.load()
B, C, H, W = 16, 128, 8, 26
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(B, C, H, W, device=dev, generator=g)
go = torch.randn(B, C, H, W, device=dev, generator=g)
yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32), torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
for name, fl in [("zero", torch.zeros(B, 2, H, W, device=dev)),
                 ("smooth2", torch.stack([2 * torch.sin(xx / 5), 2 * torch.cos(yy / 3)])[None].repeat(B, 1, 1, 1).contiguous())]:
    for v in (7, 6):
        lib.usf_set_variant(2, v)
        for nx, nf in ((True, True), (True, False), (False, True)):
            us = device_time_us(lambda: ops.warp_backward(x, fl, go, "border", nx, nf))
            print(json.dumps({"flow": name, "variant": v, "need_x": nx, "need_flow": nf, "us": round(us, 2)}), flush=True)
    lib.usf_set_variant(2, -1)
