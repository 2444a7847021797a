"""Device time of every d=4 correlation tile variant at the decoder's batch-16
sites: backward (usf_set_variant(1, i)), plain and with the sign-mask LeakyReLU
derivative, and with --fwd the forward (usf_set_variant(0, i)).

Usage (GPU box): python tools/bwd_variant_sweep.py [--fwd] [--out gpurun_out/bwd_variants.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_us, site_launcher  # noqa: E402

SITES = [(16, 32, 64, 208), (16, 64, 32, 104), (16, 96, 16, 52), (16, 128, 8, 26)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/bwd_variants.json")
    ap.add_argument("--fwd", action="store_true")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    vop = 0 if a.fwd else 1
    n = lib.usf_set_variant(vop, -1)
    res = []
    for op in (("corr_fwd",) if a.fwd else ("corr_bwd", "corr_bwd_leaky")):
        for shape in SITES:
            fn = site_launcher(op, shape if a.fwd else shape + (True, True), dev)
            for v in [-1] + list(range(n)):
                lib.usf_set_variant(vop, v)
                us = device_time_us(fn)
                res.append({"op": op, "shape": list(shape), "variant": v, "us": round(us, 2)})
                print(op, shape, v, f"{us:.2f}", flush=True)
    lib.usf_set_variant(vop, -1)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
