"""Device time of selected hot-path call sites at PWCLite's B=8 KITTI shapes
(graph-replayed launches, HIP events; unsamflow_amd.kernel_timer), with the
algorithmic GB/s and HBM fraction of each.

Usage (GPU box): python tools/sitebench.py [--ops photo_fwd_grad,photo_bwd,...]
                 [--out gpurun_out/sitebench.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_us, site_launcher  # noqa: E402

KITTI = [(192, 4, 13), (128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]
SCALES = [(256 >> i, 832 >> i) for i in range(4)]
DB = int(os.environ.get("SITEBENCH_DECODER_B", "16"))  # decoder sites: both with_bk directions stacked


def site_list(ops):
    out = []
    for op in ops:
        if op in ("corr_fwd", "corr_fwd_leaky"):
            out += [(op, (DB, C, H, W)) for C, H, W in KITTI]
        elif op in ("corr_bwd", "corr_bwd_leaky"):
            out += [(op, (DB, C, H, W, True, True)) for C, H, W in KITTI]
        elif op == "warp_fwd":
            out += [(op, (DB, C, H, W, "border")) for C, H, W in KITTI[1:]]
        elif op == "warp_bwd":
            out += [(op, (DB, C, H, W, "border", True, True)) for C, H, W in KITTI[1:]]
        elif op in ("photo_fwd", "photo_fwd_grad", "photo_pair", "photo_pair_grad"):
            out += [(op, (8, 3, H, W, "border")) for H, W in SCALES]
        elif op == "photo_bwd":
            out += [(op, (8, 2, H, W)) for H, W in SCALES]
        elif op in ("occ_bwd", "occ_vis_pair"):
            out += [(op, (8, 1, 256, 832))]
        elif op in ("convex_up", "convex_up_bwd"):
            out += [(op, (DB, H, W, 4)) for _, H, W in KITTI]
        elif op == "area_pyramid":
            out += [(op, (8, 3, 256, 832))]
        elif op in ("upsample", "upsample_bwd"):
            out += [(op, (8, 2, H, W, 2)) for _, H, W in KITTI[:4]]
        else:
            raise SystemExit(f"unknown op {op}")
    return out


def alg_bytes(op, key):
    if op == "photo_bwd":
        B, ndir, H, W = key
        return 4 * B * H * W * 6 * ndir
    if op in ("convex_up", "convex_up_bwd"):
        B, H, W, f = key  # flow + mask read, out written; backward adds grad_out, grad_flow, grad_mask
        ff = f * f
        return 4 * B * H * W * ((2 + 11 * ff) if op == "convex_up" else (4 + 20 * ff))
    B, C, H, W = key[:4]
    if op == "corr_fwd":
        return 4 * B * H * W * (2 * C + 81)
    if op == "corr_fwd_leaky":  # + the sign mask written
        return 4 * B * H * W * (2 * C + 81) + 8 * _lib.load().usf_corr_act_mask_words(B, H, W, 4)
    if op == "corr_bwd":
        return 4 * B * H * W * (81 + 4 * C)
    if op == "corr_bwd_leaky":  # + the derivative's input: the sign mask, else the activated output
        lib = _lib.load()
        words = lib.usf_corr_act_mask_words(B, H, W, 4) if lib.usf_corr_fwd_workspace(B, C, H, W, 4) == 0 else 0
        return 4 * B * H * W * (81 + 4 * C) + (8 * words if words else 4 * B * H * W * 81)
    if op == "warp_fwd":
        return 4 * B * H * W * (2 * C + 2)
    if op == "warp_bwd":
        return 4 * B * H * W * (3 * C + 4)
    if op == "photo_fwd":
        return 4 * B * H * W * (2 * C + 3)
    if op == "photo_fwd_grad":
        return 4 * B * H * W * (2 * C + 7)
    if op in ("photo_pair", "photo_pair_grad"):  # each input read once (ops.photometric_loss_pair)
        return 4 * B * H * W * (2 * C + 4 + 2 + (8 if op == "photo_pair_grad" else 0))
    if op == "occ_bwd":
        return 4 * B * H * W * 3
    if op == "occ_vis_pair":
        return 4 * B * H * W * 6
    if op == "upsample":
        return 4 * B * C * H * W * 5  # read x, write the 4x larger output
    if op == "upsample_bwd":
        return 4 * B * C * H * W * 5
    if op == "area_pyramid":
        return int(4 * B * C * H * W * (1 + 1 / 4 + 1 / 16 + 1 / 64))
    raise KeyError(op)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="photo_pair,photo_pair_grad,photo_bwd")
    ap.add_argument("--out", default="gpurun_out/sitebench.json")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda:0")
    rows = []
    for i, (op, key) in enumerate(site_list(a.ops.split(","))):
        us = device_time_us(site_launcher(op, key, dev, seed=i))
        nb = alg_bytes(op, key)
        row = {"op": op, "shape": list(key), "device_us": round(us, 2), "bytes": nb,
               "gbps": round(nb / us / 1e3, 1), "hbm_frac": round(nb / us / 1e3 / 8000.0, 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
