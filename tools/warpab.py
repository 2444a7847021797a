"""A/B of the warp backward's grad_x paths (usf_set_variant(2, v); -1 = the
default) at the decoder's batch-16 sites, on three flow fields: zero, the
smooth +-2 px field of kernel_timer.site_launcher, and a +-8 px field.
Device time (graph replay), plus the oracle-free agreement of each variant
with the default. Usage (GPU box): python tools/warpab.py [--out ...]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_us, warp_bytes  # noqa: E402

KITTI = [(128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]


def flows(B, H, W, dev, g):
    yy = torch.linspace(0, 6.2832, H, device=dev).view(1, 1, H, 1)
    xx = torch.linspace(0, 6.2832, W, device=dev).view(1, 1, 1, W)
    ph = torch.rand(B, 2, 1, 1, device=dev, generator=g) * 6.2832
    base = (torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)).contiguous()
    # shift: a large smooth motion (about 1/8 of the width plus the +-2 px field,
    # so a border strip maps outside the image and clamps onto the edge cells)
    shift = base.clone()
    shift[:, 0] += W / 8.0
    shift[:, 1] -= H / 16.0
    return {"zero": torch.zeros(B, 2, H, W, device=dev), "pm2": base, "pm8": (4 * base).contiguous(),
            "shift": shift.contiguous()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/warpab.json")
    ap.add_argument("--variants", default="-1,5,0")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    res = []
    for C, H, W in KITTI:
        B = a.batch
        g = torch.Generator(device=dev).manual_seed(C)
        x = torch.rand(B, C, H, W, device=dev, generator=g)
        go = torch.randn(B, C, H, W, device=dev, generator=g)
        for fname, fl in flows(B, H, W, dev, g).items():
            ref = None
            for v in [int(t) for t in a.variants.split(",")]:
                lib.usf_set_variant(2, v)
                gx, gf = ops.warp_backward(x, fl, go, "border")
                if ref is None:
                    ref = (gx, gf)
                err = max(float((gx - ref[0]).abs().max()), float((gf - ref[1]).abs().max()))
                us = device_time_us(lambda: ops.warp_backward(x, fl, go, "border"))
                nb = warp_bytes(B, C, H, W, True)
                row = dict(shape=[B, C, H, W], flow=fname, variant=v, us=round(us, 2), gbps=round(nb / us / 1e3, 1),
                           hbm_frac=round(nb / us / 8e6, 4), maxdiff_vs_first=err)
                res.append(row)
                print(json.dumps(row), flush=True)
            lib.usf_set_variant(2, -1)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
