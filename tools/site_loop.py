"""Launch selected hot-path call sites N times each (eager, on synthetic inputs)
for rocprofv3 --kernel-trace --stats: per-kernel device durations without the
graph-replay harness. Sites as tools/sitebench.py names them.

Usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run -- \
    python3 tools/site_loop.py --ops corr_fwd_leaky --levels 0,1 [--n 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.sitebench import site_list  # noqa: E402
from unsamflow_amd.kernel_timer import site_launcher  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="corr_fwd_leaky")
    ap.add_argument("--levels", default="0,1,2,3,4")
    ap.add_argument("--n", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lv = [int(x) for x in a.levels.split(",")]
    sites = site_list(a.ops.split(","))
    for i, (op, key) in enumerate(sites):
        if op.startswith(("corr", "warp", "convex")) and (i % 5) not in lv:
            continue
        f = site_launcher(op, key, dev, seed=i)
        for _ in range(a.n):
            f()
        torch.cuda.synchronize()
        print(op, key, flush=True)


if __name__ == "__main__":
    main()
