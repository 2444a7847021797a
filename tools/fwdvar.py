"""Device time of selected correlation-forward variants (usf_set_variant(0, i))
at given shapes, each checked against the default dispatch first.

Usage (GPU box): python tools/fwdvar.py --variants -1,8,9,13 [--shapes 8x128x32x104,...] [--bwd]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_us  # noqa: E402

SHAPES = "8x128x32x104,2x32x64x128,16x96x16x52,16x64x32x104,16x32x64x208"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--shapes", default=SHAPES)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--out", default="gpurun_out/fwdvar.json")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    op = 1 if a.bwd else 0
    rows = []
    for sh in a.shapes.split(","):
        B, C, H, W = (int(v) for v in sh.split("x"))
        g = torch.Generator(device=dev).manual_seed(C + H)
        x1 = torch.randn(B, C, H, W, device=dev, generator=g)
        x2 = torch.randn(B, C, H, W, device=dev, generator=g)
        go = torch.randn(B, 81, H, W, device=dev, generator=g)
        fn = (lambda: ops.corr_backward(x1, x2, go, 4)) if a.bwd else (lambda: ops.corr_forward(x1, x2, 4))
        lib.usf_set_variant(op, -1)
        ref = fn()
        for v in (int(t) for t in a.variants.split(",")):
            lib.usf_set_variant(op, v)
            try:
                o = fn()
                torch.cuda.synchronize()
            except RuntimeError as e:
                print(json.dumps({"shape": sh, "variant": v, "error": str(e)[:80]}), flush=True)
                continue
            if a.bwd:
                err = max((o[0] - ref[0]).abs().max().item(), (o[1] - ref[1]).abs().max().item())
            else:
                err = (o - ref).abs().max().item()
            us = device_time_us(fn)
            row = {"shape": sh, "variant": v, "us": round(us, 2), "maxerr": err}
            rows.append(row)
            print(json.dumps(row), flush=True)
        lib.usf_set_variant(op, -1)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
