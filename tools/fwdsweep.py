"""Forward correlation variant sweep at the decoder's batch-16 sites and the
SURVEY configs: warm (graph replay) and cold (read-flushed) device time of every
usf_set_variant(0, i) candidate, outputs checked against the default's.
Usage (GPU box): python tools/fwdsweep.py [--out gpurun_out/fwdsweep.json]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_cold_us, device_time_us, site_launcher  # noqa: E402

SITES = [("corr_fwd_leaky", (16, 32, 64, 208)), ("corr_fwd_leaky", (16, 64, 32, 104)),
         ("corr_fwd_leaky", (16, 96, 16, 52)), ("corr_fwd", (8, 128, 32, 104)), ("corr_fwd", (2, 32, 64, 128))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/fwdsweep.json")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n = lib.usf_set_variant(0, -1)
    res = []
    for op, key in SITES:
        fn = site_launcher(op, key, dev)
        for v in [-1] + list(range(n)):
            lib.usf_set_variant(0, v)
            try:
                warm = device_time_us(fn, reps=20, iters=10)
                cold = device_time_cold_us(fn)
            finally:
                lib.usf_set_variant(0, -1)
            res.append(dict(op=op, shape=list(key), variant=v, warm_us=round(warm, 2), cold_us=round(cold, 2)))
            print(json.dumps(res[-1]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
