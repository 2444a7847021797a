#!/usr/bin/env python3
"""Benchmark: image-pairs/sec of one PWCLite training step, KITTI 832x256, d=4.

A step (unsamflow_amd.harness.TrainStep) is the reference trainer's step:
PWCLite fwd with_bk (both directions stacked on the batch: 5 correlation + 4
decoder-warp calls at batch 16 through the HIP library; --per-direction: the
reference's two batch-8 passes) -> unFlowLoss (8 loss warps) -> backward ->
clip_grad_norm_ -> Adam ->
OneCycleLR, on B=8 synthetic U[0,1) frame pairs per GPU (kitti_base.json),
random-init weights. N>1: one process per GPU, DDP over RCCL ("nccl"), B=8
per rank (weak scaling); under torchrun the ranks come from its environment,
otherwise ``--gpus N`` starts the N rank processes itself (launch_ranks).

Output: ONE JSON line on rank 0 with the driver's contract fields plus
* ``roofline`` — the dominant hot-path call site (largest summed time per
  step): algorithmic bytes per launch / its mean launch
  duration, measured with HIP events on the launch stream around every
  library launch INSIDE the timed region (unsamflow_amd.kernel_timer); with
  USF_ROCTX=1 each launch is also a roctx range, so ``rocprofv3 --kernel-trace
  --stats --kernel-rename --marker-trace`` lists the same site as one row
  (tools/roofline_check.py compares the two);
* ``levels`` — per call site (op, level shape): in-step mean us (timed
  region) and device us of graph-replayed launches on synthetic inputs of
  that shape, GB/s, HBM fraction;
* ``cpu_baseline`` — the oracle's torch-CPU restatement of the same step
  (correlation_native-style correlation + grid_sample warp) on the host cores,
  rank 0 at N=1 only, bounded sample; plus SURVEY.md §8d's config-1 / config-2
  correlation fwd/bwd times on the CPU oracle;
* ``survey_configs`` — the same two correlation configs on the GPU kernels;
* ``roofline.copy_ceiling_gbps`` — a measured device-copy (STREAM-copy) rate
  on this box, and ``roofline.traffic`` — HBM bytes per launch of the roofline
  kernel from the committed rocprofv3 PMC passes (profiles/*_pmc_traffic.json,
  tools/pmc_traffic.py) when they cover that kernel and shape.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                       [--config kitti|sintel_mf] [--no-cpu-baseline]
       python bench.py --device cpu --gpus 2 ...   (launcher test on gloo, tests/)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import glob  # noqa: E402
import re  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md); ~6300 measured copy
CONFIGS = {
    "kitti": dict(H=256, W=832, workload="PWCLite fwd(with_bk)+unFlowLoss+bwd+Adam, KITTI 832x256, d=4"),
    "sintel_mf": dict(H=448, W=1024, workload="PWCLite+mask-feature corr fwd(with_bk)+unFlowLoss+bwd+Adam, Sintel 1024x448, d=4"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU (kitti_base.json train.batch_size)")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="kitti")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=10,
                    help="timed CPU steps (each timed on its own: the spread is reported)")
    ap.add_argument("--cpu-batch", type=int, default=8,
                    help="CPU baseline batch: the GPU's per-rank B=8 (BASELINE.md 3)")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the graph-replay device times (keeps a rocprofv3 run to real steps only)")
    ap.add_argument("--cudnn-benchmark", action="store_true",
                    help="MIOpen find-mode tuning of the convolutions (slow first steps)")
    ap.add_argument("--per-direction", action="store_true",
                    help="run with_bk as the reference's two batch-B passes instead of one batch-2B pass "
                         "(PWCLite.batch_directions = False)")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu: launcher/plumbing test only (gloo, the cpu_baseline step with the oracle ops "
                         "as the checker's stand-in; never a measurement)")
    ap.add_argument("--hw", type=int, nargs=2, metavar=("H", "W"), default=None,
                    help="frame size override (tests; the metric is KITTI 256x832)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step from HIP graphs (harness.GraphedTrainStep); measured equal to "
                         "eager at N=1 (the step is GPU-bound), so eager is the default")
    return ap.parse_args()


def cfg_for(name):
    from unsamflow_amd.config import kitti_base, sintel_mf

    return kitti_base() if name == "kitti" else sintel_mf()


def kernel_report(summary, device, steps, replay=True):
    """Per call site: in-step time (events around each launch of an untimed pass
    of the same step), device time of graph-replayed launches, algorithmic GB/s
    and HBM fraction; plus the roofline of the dominant site (by in-step time),
    whose mean main() then replaces by the timed region's own."""
    from unsamflow_amd.kernel_timer import device_time_cold_us, device_time_us, site_launcher, site_name

    rows, per_op = [], {}
    best = best_dev = None
    for i, ((op, key), a) in enumerate(summary.items()):
        calls = a["n"] / max(1, steps)
        us = a["mean_us"]
        row = {
            "op": op, "shape": list(key), "site": site_name(op, key), "calls_per_step": calls,
            "in_step_us": round(us, 2), "bytes": a["bytes"],
            "hbm_frac_in_step": round(a["bytes"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
        }
        if replay:
            # the per-level HBM fraction uses the COLD device time (read-flushed
            # caches before every launch: inputs come from HBM, as in the step for
            # the large levels); the warm graph replay keeps L3/L4 working sets in
            # the 256 MB Infinity Cache and overstates HBM. At small
            # sites the in-step interval also holds the GPU catching up with the
            # host (2-4x rocprof at L0-L2, profiles/r01_v22_roofline_check.json).
            fn = site_launcher(op, key, device, seed=i)
            dev_us = device_time_us(fn)
            cold_us = device_time_cold_us(fn)
            del fn
            row["device_us"] = round(dev_us, 2)
            row["cold_us"] = round(cold_us, 2)
            row["gbps"] = round(a["bytes"] / (cold_us * 1e-6) / 1e9, 1)
            row["hbm_frac"] = round(a["bytes"] / (cold_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
            row["hbm_frac_warm"] = round(a["bytes"] / (dev_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
            row["tflops"] = round(a["flops"] / (cold_us * 1e-6) / 1e12, 2)
            # picked by the same (cold) time its reported fraction uses
            if best_dev is None or calls * cold_us > best_dev[0]:
                best_dev = (calls * cold_us, row)
        rows.append(row)
        per_op[op] = per_op.get(op, 0.0) + calls * us
        if best is None or calls * us > best[0]:
            best = (calls * us, row)
    row = best[1]
    nbytes, extra = row["bytes"], ""
    if row["op"] in ("corr_fwd_leaky", "corr_bwd_leaky"):
        # SURVEY 8(d)'s correlation bytes; the LeakyReLU sign mask the kernel
        # also writes / reads (18 B per pixel) is reported apart, not counted
        from unsamflow_amd.kernel_timer import corr_bytes

        B, C, H, W = row["shape"][:4]
        nbytes = corr_bytes(B, C, H, W, backward=row["op"] == "corr_bwd_leaky")
        extra = f"; excludes the sign mask ({row['bytes'] - nbytes} B per launch)"
    roof = {
        "bound": "hbm",
        "kernel": row["op"],
        "shape": row["shape"],
        "site": row["site"],
        "achieved": round(nbytes / (row["in_step_us"] * 1e-6) / 1e9, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(nbytes / (row["in_step_us"] * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
        "bytes_per_launch": nbytes,
        "mean_us": row["in_step_us"],
        "launches_timed": int(round(row["calls_per_step"] * steps)),
        "replay_us": row.get("device_us"),
        "cold_us": row.get("cold_us"),
        "traffic": None,
        "method": "algorithmic bytes (SURVEY 8d) / mean duration of the site's launches in the timed region "
                  "(HIP events on the launch stream)" + extra,
    }
    if row["op"] == "warp_bwd" and row["shape"][5]:
        roof["atomic_floor"] = atomic_floor(row["shape"], row["in_step_us"])
    if best_dev is not None:
        # the dominant site by cold device time on synthetic inputs (smooth +-2 px
        # flows): the model's own random-init flows are near zero, which
        # flatters the warp backward's scatter in-step
        d = best_dev[1]
        roof["dominant_by_device"] = {"site": d["site"], "device_us": d["device_us"], "cold_us": d["cold_us"],
                                      "frac": d["hbm_frac"], "us_per_step": round(best_dev[0], 1)}
    return rows, roof, {k: round(v, 1) for k, v in per_op.items()}


def atomic_floor(shape, mean_us):
    """The warp backward's grad_x scatter is bound by fp32 atomic throughput:
    >= 2 atomics per (pixel, channel) after the wave's run merging (north and
    south corner rows), at the rate tools/probes/atomic_probe.hip measured on the
    box (profiles/r01_atomic_probe.json). Returns that floor and the site's
    fraction of it."""
    path = os.path.join(REPO, "profiles", "r01_atomic_probe.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        probe = json.load(f)
    B, C, H, W = shape[:4]
    n = 2 * B * C * H * W
    gops = max(probe["contig_2_gops"], probe["reuse2_gops"])
    floor_us = n / (gops * 1e9) * 1e6
    return {"atomics_per_launch_min": n, "atomic_rate_gops": gops, "floor_us": round(floor_us, 2),
            "frac_of_floor": round(floor_us / mean_us, 4), "source": "profiles/r01_atomic_probe.json"}


SURVEY_CONFIGS = {"cfg1": (2, 32, 64, 128), "cfg2": (8, 128, 32, 104)}
# a `levels` row: call site, launches per step, algorithmic bytes per launch, in-step
# mean us, warm graph-replay us, cold (read-flushed) us, HBM fraction from the cold
# time (the HBM-honest one), HBM fraction from the warm replay
LEVEL_FIELDS = ["site", "calls_per_step", "bytes", "in_step_us", "device_us", "cold_us", "hbm_frac", "hbm_frac_warm"]


def copy_ceiling_gbps(device, mib=512, reps=10):
    """Measured device-to-device copy rate (read + write bytes / time) of the
    library's float4 STREAM copy (usf_stream_copy_f32; MI355X_MICROARCH.md
    measures 6.29 TB/s this way, torch's copy_ reached only 4.7-5.3)."""
    from unsamflow_amd import _lib

    lib = _lib.load()
    a = torch.ones(mib * 1024 * 1024 // 4, device=device)
    b = torch.empty_like(a)
    stream = _lib.stream_handle(device)

    def copy():
        _lib.check(lib.usf_stream_copy_f32(a.data_ptr(), b.data_ptr(), a.numel(), stream), "usf_stream_copy_f32")

    copy()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        copy()
    e1.record()
    e1.synchronize()
    sec = e0.elapsed_time(e1) / 1e3 / reps
    del a, b
    return round(2 * mib * 1024 * 1024 / sec / 1e9, 1)


def pmc_traffic(op, shape):
    """HBM bytes per launch of (op, shape) from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, tools/pmc_traffic.py) measured on THIS build:
    a summary whose build_id differs from the loaded library's usf_build_id is
    never used -- a changed kernel must not inherit an old figure.
    Returns (bytes or None, source file or None, note)."""
    from unsamflow_amd import _lib

    def natural(path):  # r01_v12 after r01_v9
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    bid = _lib.build_id()
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), key=natural)
    for path in reversed(files):
        with open(path) as f:
            data = json.load(f)
        if data.get("build_id") != bid:
            continue
        for site in data.get("sites", []):
            if site["op"] == op and list(site["shape"]) == list(shape):
                return site["traffic_bytes"], os.path.relpath(path, REPO), f"build {bid}"
        return None, os.path.relpath(path, REPO), f"build {bid}: the summary does not cover this site"
    return None, None, f"no committed PMC summary of build {bid} (profiles/*_pmc_traffic.json)"


def survey_configs_gpu(device):
    from unsamflow_amd.kernel_timer import device_time_us, site_launcher

    from unsamflow_amd.kernel_timer import corr_bytes, device_time_cold_us

    out = {}
    for name, (B, C, H, W) in SURVEY_CONFIGS.items():
        ff = site_launcher("corr_fwd", (B, C, H, W), device)
        fb = site_launcher("corr_bwd", (B, C, H, W, True, True), device)
        f, b = device_time_us(ff), device_time_us(fb)
        fc, bc = device_time_cold_us(ff), device_time_cold_us(fb)
        nf, nb = corr_bytes(B, C, H, W), corr_bytes(B, C, H, W, backward=True)
        def frac(nbytes, us):
            return round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 3)

        # *_hbm_frac from the cold (read-flushed) time, as the `levels` rows;
        # *_hbm_frac_warm from the warm graph replay (inputs in the Infinity Cache)
        out[name] = {"shape": [B, C, H, W], "fwd_us": round(f, 2), "bwd_us": round(b, 2),
                     "fwd_cold_us": round(fc, 2), "bwd_cold_us": round(bc, 2),
                     "fwd_hbm_frac": frac(nf, fc), "bwd_hbm_frac": frac(nb, bc),
                     "fwd_hbm_frac_warm": frac(nf, f), "bwd_hbm_frac_warm": frac(nb, b)}
    return out


def survey_configs_cpu():
    """SURVEY §8d configs on the CPU oracle (correlation_native restatement, autograd bwd)."""
    from oracle.corr import OracleCorrelation

    corr = OracleCorrelation(4)
    out = {}
    for name, (B, C, H, W) in SURVEY_CONFIGS.items():
        g = torch.Generator().manual_seed(0)
        x1 = torch.randn(B, C, H, W, generator=g, requires_grad=True)
        x2 = torch.randn(B, C, H, W, generator=g, requires_grad=True)
        go = torch.randn(B, 81, H, W, generator=g)
        corr(x1, x2).backward(go)  # warm both directions
        x1.grad = x2.grad = None
        t0 = time.perf_counter()
        y = corr(x1, x2)
        t1 = time.perf_counter()
        y.backward(go)
        t2 = time.perf_counter()
        out[name] = {"shape": [B, C, H, W], "fwd_ms": round((t1 - t0) * 1e3, 2),
                     "bwd_ms": round((t2 - t1) * 1e3, 2)}
    return out


KITTI_LEVELS = [(192, 4, 13), (128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]


def corr_levels_cpu(B=8):
    """per-level KITTI correlation fwd / bwd (both grads) ms at
    B=8 on the CPU oracle (correlation_native.py:13-23 restated, autograd bwd)."""
    from oracle.corr import OracleCorrelation

    corr = OracleCorrelation(4)
    out = []
    for C, H, W in KITTI_LEVELS:
        g = torch.Generator().manual_seed(C)
        x1 = torch.randn(B, C, H, W, generator=g, requires_grad=True)
        x2 = torch.randn(B, C, H, W, generator=g, requires_grad=True)
        go = torch.randn(B, 81, H, W, generator=g)
        corr(x1, x2).backward(go)
        x1.grad = x2.grad = None
        t0 = time.perf_counter()
        y = corr(x1, x2)
        t1 = time.perf_counter()
        y.backward(go)
        t2 = time.perf_counter()
        out.append({"shape": [B, C, H, W], "fwd_ms": round((t1 - t0) * 1e3, 2), "bwd_ms": round((t2 - t1) * 1e3, 2)})
    return out


def cpu_baseline(args, cfg_name):
    """Oracle (torch-CPU restatement) PWCLite step on the host cores, bounded."""
    from oracle.torch_ref import OracleCorrelation, oracle_flow_warp, oracle_occu_mask_backward
    from unsamflow_amd.harness import TrainStep, synthetic_pair

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    c = CONFIGS[cfg_name]
    step = TrainStep(cfg_for(cfg_name), "cpu", corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                     occ_backward_fn=oracle_occu_mask_backward, fused_adam=False)
    img1, img2, s1, s2 = synthetic_pair(args.cpu_batch, c["H"], c["W"], "cpu", with_seg=cfg_name != "kitti")
    step(img1, img2, s1, s2)  # warmup
    per = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        step(img1, img2, s1, s2)
        per.append(time.perf_counter() - t0)
    dt = sum(per)
    rates = sorted(args.cpu_batch / t for t in per)
    mean = sum(rates) / len(rates)
    spread = {"steps": len(rates), "min": round(rates[0], 4), "median": round(rates[len(rates) // 2], 4),
              "max": round(rates[-1], 4),
              "std": round((sum((r - mean) ** 2 for r in rates) / max(1, len(rates) - 1)) ** 0.5, 4)}
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    configs = survey_configs_cpu()
    return {
        "value": round(args.cpu_batch * args.cpu_steps / dt, 4),
        "per_step_pairs_per_s": spread,
        "survey_configs": configs,
        "corr_levels": corr_levels_cpu(),
        "unit": "image-pairs/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{args.cpu_steps} steps (each timed; spread in per_step_pairs_per_s) x B={args.cpu_batch} "
                  f"({c['W']}x{c['H']}) of the same train step on CPU "
                  f"with the oracle restatement (oracle/torch_ref.py) for corr+warp+occlusion, after 1 warmup step; "
                  f"{dt:.1f} s; {model}",
    }


def _free_port():
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """--gpus N > 1 without a torch.distributed environment: start N rank
    processes of this script (one per GPU, RANK = LOCAL_RANK = r, rendezvous on
    127.0.0.1) and wait for them, as the reference's trainer spawns its own
    world (train.py:228-234, mp.spawn(main_ddp, nprocs=world_size)). Called
    before anything touches the GPU; the children are fresh processes (no exec
    from this one). A rank that fails ends the others."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.terminate()
            time.sleep(0.2)
    finally:  # the parent interrupted or failing: no orphaned rank keeps its GPU or the port
        for q in live:
            q.terminate()
        for q in live:
            try:
                q.wait(timeout=10)
            except subprocess.TimeoutExpired:
                q.kill()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        import signal

        # SIGTERM to the launcher ends its ranks too (launch_ranks' finally)
        signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    distributed = world > 1
    on_gpu = args.device == "cuda"
    if on_gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
        torch.set_num_threads(max(1, min(4, os.cpu_count() or 1)))
    if distributed:
        if on_gpu:
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)

    from unsamflow_amd.harness import GraphedTrainStep, TrainStep, broadcast_params, synthetic_pair
    from unsamflow_amd.kernel_timer import KernelTimer

    c = dict(CONFIGS[args.config])
    if args.hw:
        c["H"], c["W"] = args.hw
    cfg = cfg_for(args.config)
    if on_gpu:
        from unsamflow_amd import _lib

        _lib.load()  # fail loudly if the HIP library is missing
        use_graph = args.graph
        # graph mode: the whole step is captured once and replayed (harness.GraphedTrainStep);
        # data parallel = one all-reduce of the flat gradient buffer between the two graphs
        step = TrainStep(cfg, device, ddp=distributed and not use_graph, seed=42 + rank, capturable=use_graph)
    else:
        # launcher test only: the cpu_baseline step (oracle ops) under gloo DDP
        from oracle.torch_ref import OracleCorrelation, oracle_flow_warp, oracle_occu_mask_backward

        use_graph = False
        step = TrainStep(cfg, device, ddp=distributed, seed=42, corr_module=OracleCorrelation(4),
                         warp_fn=oracle_flow_warp, occ_backward_fn=oracle_occu_mask_backward, fused_adam=False)
    step.module.batch_directions = not args.per_direction
    img1, img2, s1, s2 = synthetic_pair(args.batch, c["H"], c["W"], device, seed=42 + rank,
                                        with_seg=args.config != "kitti")
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)

    if use_graph:
        if distributed:
            broadcast_params(step.module)
        gstep = GraphedTrainStep(step, img1, img2, s1, s2, warmup=max(3, args.warmup))
        for _ in range(2):
            gstep()
        run = gstep
    else:
        for i in range(args.warmup):
            step(img1, img2, s1, s2)
        run = lambda: step(img1, img2, s1, s2)  # noqa: E731
    sync()

    # eager: every hot-path launch's in-step time from an untimed pass of the same
    # step (two event records around each launch cost ~0.3 ms of a 40 ms step,
    # tools/kt_overhead.py); inside the timed region only the dominant call site
    # (the roofline kernel) carries its events. Graph replays carry no host code,
    # so their per-site times come from the eager pass after the timed region.
    site_pass = None
    roof_site = None
    if on_gpu and not use_graph:
        with KernelTimer() as site_pass:
            for _ in range(max(3, min(args.steps, 10))):
                run()
            sync()
        per_site = site_pass.summary()
        if per_site:
            n_pass = max(3, min(args.steps, 10))
            roof_site = max(per_site.items(), key=lambda kv: kv[1]["n"] / n_pass * kv[1]["mean_us"])[0]
    if distributed:
        dist.barrier()
    sync()
    if on_gpu and not use_graph:
        step.phase_events = []  # (start, after backward, end) device events per timed step
    with KernelTimer(enabled=on_gpu and not use_graph and roof_site is not None,
                     only={roof_site}) as kt:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = run()
        sync()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if use_graph:
        # per-site kernel times: the same step run eagerly for K steps with HIP
        # events around every library launch (kernel durations do not depend on
        # how the launch was issued; rocprofv3 of the replays cross-checks them)
        sync()
        with KernelTimer() as kt:
            for _ in range(args.steps):
                step(img1, img2, s1, s2)
            sync()
    phases = None
    if step.phase_events:
        # fwd(with_bk) + unFlowLoss + backward, and the optimizer
        # step (clip_grad_norm_ + Adam + OneCycleLR) reported apart; device time
        # between events recorded on the step's stream (max over ranks below)
        fb = sum(e[0].elapsed_time(e[1]) for e in step.phase_events) / len(step.phase_events)
        op = sum(e[1].elapsed_time(e[2]) for e in step.phase_events) / len(step.phase_events)
        step.phase_events = None
        phases = [fb, op]
    if distributed:
        t = torch.tensor([elapsed] + (phases or [0.0, 0.0]), device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t[0].item()
        if phases:
            phases = [t[1].item(), t[2].item()]
    loss_val = float(loss.item())

    rows = roof = per_op_us = gpu_configs = None
    if on_gpu:
        if site_pass is not None:
            # per-site rows from the untimed pass; the roofline site's mean from
            # the timed region itself (its launches only were bracketed there)
            n_pass = max(3, min(args.steps, 10))
            rows, roof, per_op_us = kernel_report(site_pass.summary(), device, n_pass, replay=not args.no_replay)
            timed_site = kt.summary().get(roof_site)
            if timed_site and (roof["kernel"], tuple(roof["shape"])) == roof_site:
                us = timed_site["mean_us"]
                roof["site_pass_mean_us"] = roof["mean_us"]
                roof["mean_us"] = round(us, 2)
                roof["achieved"] = round(roof["bytes_per_launch"] / (us * 1e-6) / 1e9, 1)
                roof["frac"] = round(roof["bytes_per_launch"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
                roof["launches_timed"] = timed_site["n"]
        else:
            rows, roof, per_op_us = kernel_report(kt.summary(), device, args.steps, replay=not args.no_replay)
        roof["copy_ceiling_gbps"] = copy_ceiling_gbps(device)
        roof["frac_of_copy"] = round(roof["achieved"] / roof["copy_ceiling_gbps"], 4)
        traffic, src, note = pmc_traffic(roof["kernel"], roof["shape"])
        roof["traffic"] = traffic
        roof["traffic_source"] = src
        roof["traffic_note"] = note
        gpu_configs = None if args.no_replay else survey_configs_gpu(device)

    cpu = None
    if on_gpu and rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, args.config)

    if rank == 0:
        pairs = args.batch * world * args.steps
        value = pairs / elapsed
        out = {
            "metric": "image-pairs/sec PWCLite fwd+bwd, KITTI 832x256 d=4" if args.config == "kitti"
            else "image-pairs/sec PWCLite+mask-corr fwd+bwd, Sintel 1024x448 d=4",
            "value": round(value, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic U[0,1) frame pairs, random-init PWCLite weights",
            "execution": "hip-graph replay of the captured step" if use_graph else "eager",
            "config": {
                "workload": c["workload"],
                "global_batch": args.batch * world,
                "per_gpu_batch": args.batch,
                "image_hw": [c["H"], c["W"]],
                "max_displacement": 4,
                "parallelism": f"dp{world}",
            },
            "final_loss": round(loss_val, 6),
            # untimed steps whose every hot-path launch was bracketed (the levels rows)
            "site_pass_steps": 0 if site_pass is None else max(3, min(args.steps, 10)),
            # the step split as BASELINE.md 4 defines the metric: fwd + loss + bwd, and
            # the optimizer step (clip + Adam + scheduler) apart. ms_per_step and value
            # stay the all-in wall time of the timed region (the driver's clock)
            "phases": None if not phases else {
                "fwd_loss_bwd_ms": round(phases[0], 3), "optimizer_ms": round(phases[1], 3),
                "pairs_per_s_fwd_loss_bwd": round(args.batch * world / (phases[0] / 1e3), 3),
                "method": "HIP events on the step stream around fwd+loss+bwd and clip+Adam+OneCycleLR, "
                          "mean over the timed steps, max over ranks"},
            # per call site, one compact row each (the driver keeps the last 8 KB of
            # stdout, so the summaries below come after this list)
            "levels_fields": LEVEL_FIELDS,
            "levels": None if rows is None else [[r.get(k) for k in LEVEL_FIELDS] for r in rows],
            "hot_path_us_per_step": per_op_us,
            "survey_configs": gpu_configs,
            "cpu_baseline": cpu,
            "roofline": roof,
        }
        if not on_gpu:
            out["device"] = "cpu (launcher test: oracle ops, not a measurement)"
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
