"""Correlation variant sweep at the decoder's batch-16 sites and the SURVEY
configs: warm (graph replay) and cold (read-flushed) device time of each
usf_set_variant(op, i) candidate (op 0: forward, 1: backward; parity of every
candidate is tests/test_gpu_parity.py::test_corr_every_tile_variant_vs_oracle).
Usage (GPU box): python tools/corrsweep.py [--op bwd] [--variants=-1,3] [--out F]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_cold_us, device_time_us, site_launcher  # noqa: E402

SHAPES = [(16, 32, 64, 208), (16, 64, 32, 104), (16, 96, 16, 52), (16, 128, 8, 26), (16, 192, 4, 13),
          (8, 128, 32, 104), (2, 32, 64, 128)]


def sites(op):
    """(site op, key) per shape: the decoder's LeakyReLU forms at batch 16, the plain ops at the SURVEY configs"""
    out = []
    for s in SHAPES:
        dec = s[0] == 16
        if op == "fwd":
            out.append(("corr_fwd_leaky" if dec else "corr_fwd", s))
        else:
            out.append(("corr_bwd_leaky" if dec else "corr_bwd", s + (True, True)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", choices=["fwd", "bwd"], default="fwd")
    ap.add_argument("--out", default="gpurun_out/corrsweep.json")
    ap.add_argument("--variants", default="")  # comma-separated subset (default: all)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    vop = 0 if a.op == "fwd" else 1
    n = lib.usf_set_variant(vop, -1)
    res = []
    # ~2 s of the first site before timing anything: the first measurements of a
    # fresh process otherwise run below the steady clock (L4 backward 74 vs 70 us)
    warm = site_launcher(*sites(a.op)[0], dev)
    for _ in range(400):
        warm()
    torch.cuda.synchronize()
    for op, key in sites(a.op):
        fn = site_launcher(op, key, dev)
        vs = [int(t) for t in a.variants.split(",")] if a.variants else [-1] + list(range(n))
        for v in vs:
            lib.usf_set_variant(vop, v)
            try:
                warm = device_time_us(fn, reps=20, iters=10)
                cold = device_time_cold_us(fn)
            except RuntimeError:  # a candidate that does not take this shape (the small-image kernel)
                continue
            finally:
                lib.usf_set_variant(vop, -1)
            res.append(dict(op=op, shape=list(key[:4]), variant=v, warm_us=round(warm, 2), cold_us=round(cold, 2)))
            print(json.dumps(res[-1]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
