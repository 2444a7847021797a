"""Per-call-site timing of the HIP hot-path kernels.

Two measurements, both with HIP events on the stream the kernels are launched
on (torch's current stream — the stream ops.py hands to the library):

* ``KernelTimer`` — while active, every launch made through
  :mod:`unsamflow_amd.ops` is bracketed by two event records inside the real
  training step and its call site (op, shape, flags) is recorded. These
  in-step intervals include any time the GPU waits for the host to enqueue
  the kernel, so they bound the kernel time from above.
* ``device_time_us`` — the kernel's device time on synthetic inputs of the
  call site's shape: REPS launches captured into a HIP graph, replayed back to
  back between two events, divided by the launch count (no host gaps).

With ``USF_ROCTX=1`` every launch through :mod:`unsamflow_amd.ops` is also
wrapped in a roctx range named after its call site (``site_name``), so
``rocprofv3 --kernel-trace --stats --kernel-rename --marker-trace`` reports
one row per call site, comparable with the in-step means (tools/roofline_check.py).

Algorithmic bytes / flops per launch follow SURVEY.md §8(d): every input read
once, every output written once (halo re-reads, scratch and zero-fill
excluded).
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import os

import torch

_active: "KernelTimer | None" = None
_roctx = None


def site_name(op: str, key) -> str:
    """Stable call-site label, e.g. ``usf:warp_bwd:8x32x64x208:border:1:1``."""
    return "usf:" + op + ":" + "x".join(str(k) for k in key[:4]) + "".join(f":{k}" for k in key[4:])


def _roctx_lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        if os.environ.get("USF_ROCTX") == "1":
            for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _roctx = lib
                    break
                except OSError:
                    continue
    return _roctx


def corr_bytes(B, C, H, W, K2=81, backward=False, need1=True, need2=True):
    if not backward:
        return 4 * B * H * W * (2 * C + K2)
    n = int(need1) + int(need2)  # read g once, read x_j and write grad_i per needed grad
    return 4 * B * H * W * (K2 + 2 * n * C)


def corr_flops(B, C, H, W, K2=81, backward=False, need1=True, need2=True):
    n = (int(need1) + int(need2)) if backward else 1
    return 2 * K2 * C * B * H * W * n


def warp_bytes(B, C, H, W, backward=False, need_x=True, need_flow=True):
    if not backward:
        return 4 * B * H * W * (2 * C + 2)
    per_px = 2 + C  # flow, grad_out
    if need_flow:
        per_px += C + 2  # x, grad_flow
    if need_x:
        per_px += C  # grad_x
    return 4 * B * H * W * per_px


class KernelTimer:
    def __init__(self, time_in_step: bool = True, enabled: bool = True, only=None):
        self.time_in_step = time_in_step
        self.enabled = enabled  # False: a no-op context (nothing recorded)
        # only: a set of (op, key) call sites to bracket (None: every launch), so a
        # timed region can carry the events of one site and no others
        self.only = only
        self.records = []  # (op, key, start_event, end_event, bytes, flops)

    def __enter__(self):
        global _active
        self._prev = _active
        if self.enabled:
            _active = self
        return self

    def __exit__(self, *exc):
        global _active
        _active = self._prev
        return False

    def summary(self):
        """{(op, key): dict(n, mean_us (in-step), bytes, flops)} — call after a device sync."""
        agg = collections.OrderedDict()
        for op, key, s, e, nbytes, flops in self.records:
            a = agg.setdefault((op, key), {"n": 0, "total_us": 0.0, "bytes": nbytes, "flops": flops})
            a["n"] += 1
            if s is not None:
                a["total_us"] += s.elapsed_time(e) * 1e3
        for a in agg.values():
            a["mean_us"] = a["total_us"] / a["n"]
        return agg


@contextlib.contextmanager
def timed(op: str, key, device, nbytes: int, flops: int = 0):
    """Bracket one launch (used by ops.py)."""
    rx = _roctx_lib()
    if rx:
        rx.roctxRangePushA(site_name(op, key).encode())
    try:
        kt = _active
        if kt is None or (kt.only is not None and (op, tuple(key)) not in kt.only):
            yield
            return
        if not kt.time_in_step:
            yield
            kt.records.append((op, key, None, None, nbytes, flops))
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(device)
        s.record(stream)
        yield
        e.record(stream)
        kt.records.append((op, key, s, e, nbytes, flops))
    finally:
        if rx:
            rx.roctxRangePop()


def site_launcher(op: str, key, device, seed: int = 0):
    """A closure launching one kernel of call site (op, key) on synthetic inputs.

    Inputs: N(0,1) features / gradients, U[0,1) images, and a smooth warp flow
    of +-2 px amplitude (two low-frequency sinusoids per component: the
    magnitude and smoothness of PWCLite's flows early in training). Per-pixel
    random flows would scatter the grad_x atomics and misstate the kernel.
    """
    from . import ops

    g = torch.Generator(device=device).manual_seed(seed)
    if op == "corr_bwd_leaky":  # the decoder's site: g from a concat slice + LeakyReLU derivative
        B, C, H, W = key[:4]
        x1 = torch.randn(B, C, H, W, device=device, generator=g)
        x2 = torch.randn(B, C, H, W, device=device, generator=g)
        cat = torch.randn(B, 81 + C + 2, H, W, device=device, generator=g)
        act = torch.nn.functional.leaky_relu(torch.randn(B, 81 + C + 2, H, W, device=device, generator=g), 0.1)
        # as corr_cat runs it: the forward's sign mask where W % 4 == 0, else the dense pass
        mask = ops.corr_act_mask(B, H, W, 4, device, C=C)
        if mask is not None:
            ops.corr_forward_ex(x1, x2, 4, act[:, :81], 0.1, act_mask=mask)
        return lambda: ops.corr_backward_ex(x1, x2, cat[:, :81], 4, key[4], key[5], act_out=act[:, :81],
                                            act_mask=mask)
    if op == "corr_fwd_leaky":  # the decoder's forward: LeakyReLU into a concat slice + sign mask
        B, C, H, W = key[:4]
        x1 = torch.randn(B, C, H, W, device=device, generator=g)
        x2 = torch.randn(B, C, H, W, device=device, generator=g)
        cat = torch.empty(B, 81 + C + 2, H, W, device=device)
        mask = ops.corr_act_mask(B, H, W, 4, device, C=C)
        return lambda: ops.corr_forward_ex(x1, x2, 4, cat[:, :81], 0.1, act_mask=mask)
    if op in ("corr_fwd", "corr_bwd"):
        B, C, H, W = key[:4]
        x1 = torch.randn(B, C, H, W, device=device, generator=g)
        x2 = torch.randn(B, C, H, W, device=device, generator=g)
        if op == "corr_fwd":
            return lambda: ops.corr_forward(x1, x2, 4)
        need1, need2 = key[4], key[5]
        go = torch.randn(B, 81, H, W, device=device, generator=g)
        return lambda: ops.corr_backward(x1, x2, go, 4, need1, need2)
    if op in ("upsample", "upsample_bwd"):
        B, C, H, W, k = key[:5]
        if op == "upsample":
            f = torch.randn(B, C, H, W, device=device, generator=g)
            return lambda: ops.flow_upsample(f, k)
        go = torch.randn(B, C, H * k, W * k, device=device, generator=g)
        return lambda: ops.flow_upsample_backward(go, k)
    if op in ("convex_pyr", "convex_pyr_bwd"):  # every decoder level in one launch
        B, f = key[0], key[-1]
        hw = [(key[i], key[i + 1]) for i in range(1, len(key) - 1, 2)]
        flows = [torch.randn(B, 2, h, w, device=device, generator=g) for h, w in hw]
        masks = [torch.randn(B, 9 * f * f, h, w, device=device, generator=g) for h, w in hw]
        if op == "convex_pyr":
            return lambda: ops.convex_upsample_pyramid(flows, masks, f)
        gos = [torch.randn(B, 2, f * h, f * w, device=device, generator=g) for h, w in hw]
        return lambda: ops.convex_upsample_pyramid_backward(flows, masks, gos, f)
    if op in ("convex_up", "convex_up_bwd"):
        B, H, W, f = key
        flow = torch.randn(B, 2, H, W, device=device, generator=g)
        mask = torch.randn(B, 9 * f * f, H, W, device=device, generator=g)
        if op == "convex_up":
            return lambda: ops.convex_upsample(flow, mask, f)
        go = torch.randn(B, 2, f * H, f * W, device=device, generator=g)
        return lambda: ops.convex_upsample_backward(flow, mask, go, f)
    if op == "area_pyramid":
        img = torch.rand(*key, device=device, generator=g)
        return lambda: ops.area_pyramid(img)
    if op == "photo_bwd":
        B, ndir, H, W = key
        basis = torch.randn(B, 4 * ndir, H, W, device=device, generator=g)
        coef = torch.rand(3 * ndir, device=device, generator=g)
        gl = torch.ones(ndir, device=device)
        return lambda: ops.photo_loss_backward(basis, coef, gl)
    if op in ("photo_pyr", "photo_pyr_grad", "photo_pyr_bwd"):  # the loss scales in one launch
        B, C = key[:2]
        hw = [(key[i], key[i + 1]) for i in range(2, len(key) - (op != "photo_pyr_bwd"), 2)]
        if op == "photo_pyr_bwd":
            bases = [torch.randn(B, 8, h, w, device=device, generator=g) for h, w in hw]
            coef = torch.rand(6 * len(hw), device=device, generator=g)
            gl = torch.ones(2 * len(hw), device=device)
            return lambda: ops.photo_loss_pyramid_backward(bases, coef, gl)
        flows, i1, i2, m1, m2 = [], [], [], [], []
        for h, w in hw:
            yy = torch.linspace(0, 6.2832, h, device=device).view(1, 1, h, 1)
            xx = torch.linspace(0, 6.2832, w, device=device).view(1, 1, 1, w)
            ph = torch.rand(B, 2, 1, 1, device=device, generator=g) * 6.2832
            f2 = torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)
            flows.append(torch.cat([f2, -f2], 1).contiguous())
            i1.append(torch.rand(B, C, h, w, device=device, generator=g))
            i2.append(torch.rand(B, C, h, w, device=device, generator=g))
            m1.append((torch.rand(B, 1, h, w, device=device, generator=g) > 0.1).float())
            m2.append(m1[-1].flip(-1).contiguous())
        return lambda: ops.photo_loss_pyramid_forward(flows, i1, i2, m1, m2, key[-1], need_grad=op == "photo_pyr_grad")
    if op == "occ_vis_pair":  # both directions of the loss's masks from a [B,4,H,W] flow
        B, _, H, W = key[:4]
        yy = torch.linspace(0, 6.2832, H, device=device).view(1, 1, H, 1)
        xx = torch.linspace(0, 6.2832, W, device=device).view(1, 1, 1, W)
        ph = torch.rand(B, 2, 1, 1, device=device, generator=g) * 6.2832
        f2 = torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)
        flow4 = torch.cat([f2, -f2], 1).contiguous()
        return lambda: ops.occ_vis_pair(flow4, 0.2)
    if op in ("occ_bwd", "splat", "photo_fwd", "photo_fwd_grad", "photo_pair", "photo_pair_grad"):
        B, C, H, W = key[:4]
        yy = torch.linspace(0, 6.2832, H, device=device).view(1, 1, H, 1)
        xx = torch.linspace(0, 6.2832, W, device=device).view(1, 1, 1, W)
        ph = torch.rand(B, 2, 1, 1, device=device, generator=g) * 6.2832
        flow = (torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)).contiguous()
        if op == "occ_bwd":
            return lambda: ops.occ_backward(flow, 0.2)
        if op == "splat":
            return lambda: ops.splat_map(flow, bool(key[4]))
        pad = key[4]
        src = torch.rand(B, C, H, W, device=device, generator=g)
        tgt = torch.rand(B, C, H, W, device=device, generator=g)
        mask = (torch.rand(B, 1, H, W, device=device, generator=g) > 0.1).float()
        if op.startswith("photo_pair"):
            flow4 = torch.cat([flow, -flow], 1)
            mask2 = mask.flip(-1).contiguous()
            return lambda: ops.photo_loss_pair_forward(flow4, tgt, src, mask, mask2, pad,
                                                       need_grad=op == "photo_pair_grad")
        return lambda: ops.photo_loss_forward(src, tgt, mask, flow, pad, need_grad=op == "photo_fwd_grad")
    B, C, H, W, pad = key[:5]
    x = torch.rand(B, C, H, W, device=device, generator=g)
    yy = torch.linspace(0, 6.2832, H, device=device).view(1, 1, H, 1)
    xx = torch.linspace(0, 6.2832, W, device=device).view(1, 1, 1, W)
    ph = torch.rand(B, 2, 1, 1, device=device, generator=g) * 6.2832
    flow = (torch.sin(2 * xx + ph) + torch.cos(3 * yy - ph)).contiguous()  # [B,2,H,W], |f| <= 2
    if op == "warp_fwd":
        return lambda: ops.warp_forward(x, flow, pad)
    if op == "warp_fwd_up":  # the decoder's x2 upsampling of a coarse flow fused with the warp
        coarse = (flow[:, :, ::2, ::2] * 0.5).contiguous()
        return lambda: ops.warp_forward_up(x, coarse, pad)
    need_x, need_flow = key[5], key[6]
    go = torch.randn(B, C, H, W, device=device, generator=g)
    return lambda: ops.warp_backward(x, flow, go, pad, need_x, need_flow)


_flush = {}


def device_time_cold_us(fn, reps: int = 8, flush_mib: int = 512) -> float:
    """Mean duration of one ``fn()`` launch from cold caches (HBM-honest).

    Before every timed launch a read sweep over a ``flush_mib`` MiB scratch
    buffer (a sum into one element: reads only, so no dirty lines are written
    back during the timed launch; a write flush overshot) evicts
    the 256 MiB Infinity Cache and the L2s. Two events bracket the launch alone
    on the launch stream; the sweep runs for ~0.1 ms, long enough for the host
    to enqueue the launch before the GPU reaches it, so the interval holds no
    host gap. The outputs of the previous launch are written back during the
    sweep, not during the timed launch."""
    dev = torch.cuda.current_device()
    if dev not in _flush:
        _flush[dev] = (torch.ones(flush_mib * 1024 * 1024 // 4, device="cuda"), torch.empty((), device="cuda"))
    buf, sink = _flush[dev]
    for _ in range(2):
        fn()
    evs = []
    for _ in range(reps):
        torch.sum(buf, dim=0, out=sink)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        evs.append((s, e))
    torch.cuda.synchronize()
    times = sorted(s.elapsed_time(e) * 1e3 for s, e in evs)
    return sum(times[1:-1]) / (len(times) - 2) if len(times) > 2 else times[0]


def device_time_us(fn, reps: int = 20, iters: int = 5) -> float:
    """Mean device time of one ``fn()`` launch: REPS launches in a HIP graph, replayed."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        graph.replay()
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) * 1e3 / (iters * reps)
    del graph
    return us
