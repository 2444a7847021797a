"""A/B timing of the fused photometric pair kernel (photo.hip) at the loss's
four scales, one process per library build (USF_LIB=<path> from
tools/ab_build.py). Each row carries a hash of the outputs so the builds can
be checked for bit-identical results. Device times: graph-replayed launches
(unsamflow_amd.kernel_timer.device_time_us).

Usage (GPU box): USF_LIB=... python tools/photoab.py --out gpurun_out/photoab/x.json
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd.kernel_timer import device_time_us, site_launcher  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--variant", type=int, default=-1,
                    help="usf_set_variant(3, v): -1 the default; the library has one pair kernel "
                         "(producer/consumer), so any other value is refused")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from unsamflow_amd import _lib

    rc = _lib.load().usf_set_variant(3, a.variant)
    if rc < 0:
        sys.exit(f"usf_set_variant(3, {a.variant}) refused (rc {rc}): no such photometric variant")
    sites = [("photo_pair_grad", (8, 3, 256 >> i, 832 >> i, "border")) for i in range(4)]
    sites += [("photo_pair_grad", (8, 3, 256, 832, "zeros")), ("photo_pair", (8, 3, 256, 832, "border"))]
    rows = []
    for op, key in sites:
        fn = site_launcher(op, key, dev)
        out, basis = fn()
        torch.cuda.synchronize()
        h = hashlib.sha1(out.cpu().numpy().tobytes())
        if basis is not None:
            h.update(basis.cpu().numpy().tobytes())
        us = device_time_us(fn, reps=20, iters=10)
        rows.append({"op": op, "shape": list(key), "us": round(us, 2), "hash": h.hexdigest()[:16]})
        print(json.dumps(rows[-1]), flush=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
