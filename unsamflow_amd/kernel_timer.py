"""Optional per-launch timing of the HIP hot-path kernels with HIP events.

When enabled (``with KernelTimer() as kt: ...``), every launch made through
:mod:`unsamflow_amd.ops` is bracketed by two ``torch.cuda.Event`` records on
the stream the kernel is launched on (torch's current stream of the tensor's
device — the same stream ops.py passes to the library), tagged with the op
name, shape and the algorithmic byte / flop counts of SURVEY.md §8d. After a
device sync, :meth:`KernelTimer.summary` aggregates mean duration and
achieved GB/s per (op, shape). Disabled, it costs one global check per call.
"""
from __future__ import annotations

import collections
import contextlib

import torch

_active: "KernelTimer | None" = None


def corr_bytes(B, C, H, W, K2=81, backward=False, need1=True, need2=True):
    if not backward:
        return 4 * B * H * W * (2 * C + K2)
    # read g once, read the x each grad needs, write each grad once
    n = int(need1) + int(need2)
    return 4 * B * H * W * (K2 + 2 * n * C)


def corr_flops(B, C, H, W, K2=81, backward=False, need1=True, need2=True):
    n = (int(need1) + int(need2)) if backward else 1
    return 2 * K2 * C * B * H * W * n


def warp_bytes(B, C, H, W, backward=False, need_x=True, need_flow=True):
    if not backward:
        return 4 * B * H * W * (2 * C + 2)
    per_px = 2  # read flow
    per_px += C  # read grad_out
    if need_flow:
        per_px += C + 2  # read x, write grad_flow
    if need_x:
        per_px += C  # grad_x (read-modify-write by atomics counted once)
    return 4 * B * H * W * per_px


class KernelTimer:
    def __init__(self):
        self.records = []  # (op, key, start_event, end_event, bytes, flops)

    def __enter__(self):
        global _active
        self._prev = _active
        _active = self
        return self

    def __exit__(self, *exc):
        global _active
        _active = self._prev
        return False

    def summary(self):
        """{(op, key): dict(n, mean_us, bytes, flops, gbps, tflops)} — call after a device sync."""
        agg = collections.OrderedDict()
        for op, key, s, e, nbytes, flops in self.records:
            ms = s.elapsed_time(e)
            a = agg.setdefault((op, key), {"n": 0, "total_us": 0.0, "bytes": nbytes, "flops": flops})
            a["n"] += 1
            a["total_us"] += ms * 1e3
        for a in agg.values():
            a["mean_us"] = a["total_us"] / a["n"]
            a["gbps"] = a["bytes"] / (a["mean_us"] * 1e-6) / 1e9
            a["tflops"] = a["flops"] / (a["mean_us"] * 1e-6) / 1e12
        return agg


@contextlib.contextmanager
def timed(op: str, key, device, nbytes: int, flops: int = 0):
    """Bracket one launch (used by ops.py)."""
    kt = _active
    if kt is None:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(device)
    s.record(stream)
    yield
    e.record(stream)
    kt.records.append((op, key, s, e, nbytes, flops))
