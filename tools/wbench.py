"""Warp-backward micro-benchmark: device time of usf_warp_bwd_f32 by component
(grad_x + grad_flow, grad_x only, grad_flow only), flow field and grad_x
scatter variant, at the decoder's L4/L3 shapes (graph-replayed, HIP events).

Usage (GPU box): python tools/wbench.py [--out gpurun_out/wbench.json]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_us  # noqa: E402


def flows(B, H, W, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    yy = torch.linspace(0, 2 * math.pi, H, device=dev).view(1, 1, H, 1)
    xx = torch.linspace(0, 2 * math.pi, W, device=dev).view(1, 1, 1, W)
    ph = torch.rand(B, 2, 1, 1, device=dev, generator=g) * 2 * math.pi
    sin2 = (torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)).contiguous()
    return {
        "zero": torch.zeros(B, 2, H, W, device=dev),
        "const(0.3,0.2)": torch.tensor([0.3, 0.2], device=dev).view(1, 2, 1, 1).expand(B, 2, H, W).contiguous(),
        "sin+-2": sin2,
        "sin+-8": (4 * sin2).contiguous(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/wbench.json")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    res = []
    for (B, C, H, W) in [(16, 32, 64, 208), (16, 64, 32, 104), (16, 96, 16, 52), (16, 128, 8, 26)]:
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.rand(B, C, H, W, device=dev, generator=g)
        go = torch.randn(B, C, H, W, device=dev, generator=g)
        z = device_time_us(lambda: torch.zeros_like(x))
        res.append({"shape": [B, C, H, W], "what": "zeros_like(grad_x) alone", "us": round(z, 2)})
        print(f"{(B, C, H, W)} memset grad_x {z:.2f} us", flush=True)
        for fname, fl in flows(B, H, W, dev).items():
            for need_x, need_f in ((True, True), (True, False), (False, True)):
                # -1: lane-merged scatter (default); 1: LDS-aggregated scatter; 4: gather grad_x
                for v in ((-1, 4, 5) if need_x else (-1,)):
                    lib.usf_set_variant(2, v)
                    t = device_time_us(lambda: ops.warp_backward(x, fl, go, "border", need_x, need_f))
                    row = {"shape": [B, C, H, W], "flow": fname, "grad_x": need_x, "grad_flow": need_f,
                           "variant": v, "us": round(t, 2)}
                    res.append(row)
                    print(f"{(B, C, H, W)} flow={fname:15s} gx={need_x:d} gf={need_f:d} v={v:2d}: {t:7.2f} us", flush=True)
        lib.usf_set_variant(2, -1)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
