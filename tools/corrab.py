"""A/B timing of the correlation kernels at the decoder's call sites and the
SURVEY configs, with an fp64 torch check of every timed configuration.

One process per library build (USF_LIB=<path> picks an A/B build from
tools/ab_build.py). Times are device times (graph-replayed launches,
unsamflow_amd.kernel_timer.device_time_us).

Usage (GPU box): python tools/corrab.py [--out gpurun_out/corrab.json] [--ops fwd,bwd,leaky]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import corr_bytes, device_time_us, site_launcher  # noqa: E402

KITTI = [(192, 4, 13), (128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]
SURVEY = {"cfg1": (2, 32, 64, 128), "cfg2": (8, 128, 32, 104)}


def corr_ref64(x1, x2, d=4):
    """correlation_native.py:13-23 in fp64 on the device (the checker only)."""
    B, C, H, W = x1.shape
    p = F.pad(x2, (d, d, d, d))
    outs = [(x1 * p[:, :, i:i + H, j:j + W]).mean(1, keepdim=True)
            for i in range(2 * d + 1) for j in range(2 * d + 1)]
    return torch.cat(outs, 1)


def check_fwd(shape, dev):
    g = torch.Generator(device=dev).manual_seed(1)
    x1 = torch.randn(*shape, device=dev, generator=g)
    x2 = torch.randn(*shape, device=dev, generator=g)
    out = ops.corr_forward(x1, x2, 4)
    ref = corr_ref64(x1.double(), x2.double())
    return (out.double() - ref).abs().max().item()


def check_bwd(shape, dev):
    g = torch.Generator(device=dev).manual_seed(2)
    B, C, H, W = shape
    x1 = torch.randn(*shape, device=dev, generator=g)
    x2 = torch.randn(*shape, device=dev, generator=g)
    go = torch.randn(B, 81, H, W, device=dev, generator=g)
    g1, g2 = ops.corr_backward(x1, x2, go, 4)
    a = x1.double().requires_grad_(True)
    b = x2.double().requires_grad_(True)
    corr_ref64(a, b).backward(go.double())
    return max((g1.double() - a.grad).abs().max().item(), (g2.double() - b.grad).abs().max().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/corrab.json")
    ap.add_argument("--ops", default="fwd,bwd,leaky")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--fwd-variant", type=int, default=-1)
    ap.add_argument("--bwd-variant", type=int, default=-1)
    a = ap.parse_args()
    lib = _lib.load()
    lib.usf_set_variant(0, a.fwd_variant)
    lib.usf_set_variant(1, a.bwd_variant)
    dev = torch.device("cuda:0")
    res = []
    todo = []
    if "leaky" in a.ops:
        todo += [("corr_bwd_leaky", (a.batch, C, H, W, True, True)) for C, H, W in KITTI]
    if "fwd" in a.ops:
        todo += [("corr_fwd", (a.batch, C, H, W)) for C, H, W in KITTI]
        todo += [("corr_fwd", s) for s in SURVEY.values()]
    if "bwdk" in a.ops.split(","):  # plain backward (no LeakyReLU) at the decoder's shapes
        todo += [("corr_bwd", (a.batch, C, H, W, True, True)) for C, H, W in KITTI]
    if "bwd" in a.ops.split(","):
        todo += [("corr_bwd", (*s, True, True)) for s in SURVEY.values()]
    for op, key in todo:
        us = device_time_us(site_launcher(op, key, dev), reps=20, iters=10)
        B, C, H, W = key[:4]
        nb = corr_bytes(B, C, H, W, backward=op != "corr_fwd")
        row = dict(op=op, shape=list(key[:4]), us=round(us, 2), gbps=round(nb / us / 1e3, 1),
                   hbm_frac=round(nb / us / 8e6, 4))
        if op == "corr_fwd" and (tuple(key) in SURVEY.values() or B * C * H * W <= 8 * 128 * 32 * 104):
            row["maxerr"] = check_fwd(key, dev)
        if op == "corr_bwd":
            row["maxerr"] = check_bwd(key[:4], dev)
        res.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
