"""Is the PWCLite step host-bound? Eager step: host enqueue time vs wall time;
then the same step captured into HIP graphs (harness.GraphedTrainStep) and
replayed. Also checks that a replayed step trains like an eager one (loss of
the next step from identical starting states).

Usage (GPU box): python tools/graph_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.config import kitti_base  # noqa: E402
from unsamflow_amd.harness import GraphedTrainStep, TrainStep, synthetic_pair  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--eager-only", action="store_true")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda:0")
    img1, img2, _, _ = synthetic_pair(8, 256, 832, dev)
    res = {"tag": a.tag, "channels_last": a.channels_last}
    step = TrainStep(kitti_base(), dev, capturable=True, channels_last=a.channels_last)
    for _ in range(5):
        step(img1, img2)
    torch.cuda.synchronize()
    n = 10
    enq = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        step(img1, img2)
        enq.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    res["eager_ms_per_step"] = (time.perf_counter() - t0) / n * 1e3
    res["eager_host_enqueue_ms"] = sum(enq) / n * 1e3
    print(json.dumps(res), flush=True)
    if a.eager_only:
        return

    t0 = time.perf_counter()
    g = GraphedTrainStep(step, img1, img2, warmup=3)
    torch.cuda.synchronize()
    res["capture_s"] = time.perf_counter() - t0
    for _ in range(3):
        g()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        loss = g()
    torch.cuda.synchronize()
    res["graph_ms_per_step"] = (time.perf_counter() - t0) / n * 1e3
    res["graph_loss"] = float(loss)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
