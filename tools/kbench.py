"""Kernel micro-benchmark: device time of every tile variant of the correlation
kernels (usf_set_variant) and of the warp kernels at PWCLite's call-site shapes
(KITTI 832x256, B=8), via graph-replayed launches (unsamflow_amd.kernel_timer).
Each variant's output is checked against the default heuristic's before timing.

Usage (GPU box): python tools/kbench.py [--out gpurun_out/kbench.json] [--quick]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import corr_bytes, device_time_us, site_launcher, warp_bytes  # noqa: E402

KITTI = [(192, 4, 13), (128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/kbench.json")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ops", default="corr_fwd,corr_bwd,warp")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    B = a.batch
    res = []
    nf = lib.usf_set_variant(0, -1)
    nb = lib.usf_set_variant(1, -1)
    for (C, H, W) in KITTI:
        g = torch.Generator(device=dev).manual_seed(C)
        x1 = torch.randn(B, C, H, W, device=dev, generator=g)
        x2 = torch.randn(B, C, H, W, device=dev, generator=g)
        go = torch.randn(B, 81, H, W, device=dev, generator=g)
        if "corr_fwd" in a.ops:
            ref = ops.corr_forward(x1, x2, 4)
            for v in [-1] + list(range(nf)):
                lib.usf_set_variant(0, v)
                out = ops.corr_forward(x1, x2, 4)
                err = (out - ref).abs().max().item()
                us = device_time_us(lambda: ops.corr_forward(x1, x2, 4))
                nbytes = corr_bytes(B, C, H, W)
                res.append(dict(op="corr_fwd", shape=[B, C, H, W], variant=v, us=round(us, 2),
                                gbps=round(nbytes / us / 1e3, 1), maxerr=err))
                print(res[-1], flush=True)
            lib.usf_set_variant(0, -1)
        if "corr_bwd" in a.ops:
            r1, r2 = ops.corr_backward(x1, x2, go, 4)
            for v in [-1] + list(range(nb)):
                lib.usf_set_variant(1, v)
                g1, g2 = ops.corr_backward(x1, x2, go, 4)
                err = max((g1 - r1).abs().max().item(), (g2 - r2).abs().max().item())
                us = device_time_us(lambda: ops.corr_backward(x1, x2, go, 4))
                nbytes = corr_bytes(B, C, H, W, backward=True)
                res.append(dict(op="corr_bwd", shape=[B, C, H, W], variant=v, us=round(us, 2),
                                gbps=round(nbytes / us / 1e3, 1), maxerr=err))
                print(res[-1], flush=True)
            lib.usf_set_variant(1, -1)
        if "warp" in a.ops and H > 4:
            k = (B, C, H, W, "border")
            us = device_time_us(site_launcher("warp_fwd", k, dev))
            res.append(dict(op="warp_fwd", shape=list(k), us=round(us, 2), gbps=round(warp_bytes(B, C, H, W) / us / 1e3, 1)))
            print(res[-1], flush=True)
            k = (B, C, H, W, "border", True, True)
            for v in (-1, 0, 1, 2, 3):
                lib.usf_set_variant(2, v)
                us = device_time_us(site_launcher("warp_bwd", k, dev))
                res.append(dict(op="warp_bwd", shape=list(k), variant=v, us=round(us, 2),
                                gbps=round(warp_bytes(B, C, H, W, True) / us / 1e3, 1)))
                print(res[-1], flush=True)
            lib.usf_set_variant(2, -1)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
