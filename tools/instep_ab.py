"""Same-process A/B of the training step: alternate between library builds
(ctypes handles swapped under unsamflow_amd._lib) and/or Python-side knobs of
unsamflow_amd.ops, timing every hot-path launch inside real steps
(KernelTimer, HIP events on the launch stream), so each form is judged by its
in-step time on the same box, inputs and model state.

Usage (GPU box, repo root):
  python tools/instep_ab.py --libs main,unsamflow_amd/lib/ab/lib_x.so [--ops warp_bwd,corr_bwd_leaky]
  python tools/instep_ab.py --knob WARP_PERSIST_MAX_PIXELS=none,1000
  [--rounds 3 --steps 10 --warmup 5 --out gpurun_out/ab.json]
"""
import argparse
import ctypes
import importlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.config import kitti_base  # noqa: E402
from unsamflow_amd.harness import TrainStep, synthetic_pair  # noqa: E402
from unsamflow_amd.kernel_timer import KernelTimer, site_name  # noqa: E402


def load_handle(path):
    if path == "main":
        return _lib.load()
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name, (argtypes, restype) in _lib._SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    assert lib.usf_abi_version() == _lib.ABI_VERSION, path
    return lib


def parse_value(v):
    return None if v == "none" else int(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="main")
    ap.add_argument("--knob", default=None, help="NAME=v1,v2 (an ops module global)")
    ap.add_argument("--ops", default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    configs = []
    for lp in a.libs.split(","):
        if a.knob:
            name, _, vals = a.knob.partition("=")
            configs += [(lp, name, parse_value(v)) for v in vals.split(",")]
        else:
            configs.append((lp, None, None))
    handles = {lp: load_handle(lp) for lp in {c[0] for c in configs}}
    step = TrainStep(kitti_base(), dev, seed=42)
    img1, img2, _, _ = synthetic_pair(8, 256, 832, dev)
    only = set(a.ops.split(",")) if a.ops else None

    def use(cfg):
        lp, name, val = cfg
        torch.cuda.synchronize()
        ops.clear_persistent_workspaces()  # layouts may differ between builds
        _lib._lib = handles[lp]
        if name:  # an ops global, or module.NAME of another unsamflow_amd module
            mod, _, attr = name.rpartition(".")
            target = importlib.import_module("unsamflow_amd." + mod) if mod else ops
            setattr(target, attr, val)

    res = {c: {"ms": [], "sites": {}} for c in configs}
    for c in configs:  # warm every configuration (solver caches, allocator, workspaces)
        use(c)
        for _ in range(a.warmup):
            step(img1, img2)
    for r in range(a.rounds):
        for c in configs:
            use(c)
            step(img1, img2)
            torch.cuda.synchronize()
            with KernelTimer() as kt:
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step(img1, img2)
                torch.cuda.synchronize()
                res[c]["ms"].append((time.perf_counter() - t0) / a.steps * 1e3)
            for (op, key), s in kt.summary().items():
                if only and op not in only:
                    continue
                res[c]["sites"].setdefault(site_name(op, key), []).append(s["mean_us"])
        print(f"round {r} done", flush=True)
    out = []
    for c in configs:
        row = {"lib": c[0], "knob": c[1], "value": c[2], "ms_per_step": round(statistics.median(res[c]["ms"]), 3),
               "sites_in_step_us": {k: round(statistics.median(v), 2) for k, v in res[c]["sites"].items()}}
        out.append(row)
        print(json.dumps(row))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rounds": a.rounds, "steps": a.steps, "configs": out}, f, indent=1)


if __name__ == "__main__":
    main()
