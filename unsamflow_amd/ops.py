"""Tensor-level entry points to the HIP kernels (no autograd).

Each function validates its tensors, allocates the outputs with torch (the
caching allocator owns all memory; the library never allocates), and launches
on torch's current stream of the tensors' device. There is deliberately no
CPU path: CPU tensors raise ``RuntimeError``.
"""
from __future__ import annotations

import torch

from collections import OrderedDict

from . import _lib
from . import kernel_timer as _kt

PAD_MODES = {"zeros": _lib.PAD_ZEROS, "border": _lib.PAD_BORDER}


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _require_device_f32(name: str, t: torch.Tensor) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"unsamflow_amd: {name} is on {t.device}; the HIP kernels need tensors on a ROCm "
            "device (there is no CPU path)"
        )
    if t.dtype != torch.float32:
        raise TypeError(f"unsamflow_amd: {name} must be float32, got {t.dtype}")


def _check_out(name: str, t: torch.Tensor, shape, device) -> None:
    if tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or t.device != device or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous float32 {tuple(shape)} tensor on {device}")


def _nchw(name: str, t: torch.Tensor) -> tuple[int, int, int, int]:
    if t.dim() != 4:
        raise ValueError(f"{name} must be 4-D NCHW, got shape {tuple(t.shape)}")
    return tuple(t.shape)  # type: ignore[return-value]


def corr_forward(x1: torch.Tensor, x2: torch.Tensor, max_displacement: int,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Cost volume [B,(2d+1)^2,H,W] of x1 against x2 (correlation_native.py:13-23).

    ``out``: optional preallocated contiguous fp32 output of the right shape."""
    _require_device_f32("input1", x1)
    _require_device_f32("input2", x2)
    B, C, H, W = _nchw("input1", x1)
    if x2.shape != x1.shape:
        raise ValueError(f"input2 shape {tuple(x2.shape)} != input1 shape {tuple(x1.shape)}")
    if x2.device != x1.device:
        raise ValueError("input1 and input2 are on different devices")
    d = int(max_displacement)
    K = 2 * d + 1
    x1c, x2c = x1.contiguous(), x2.contiguous()
    if out is None:
        out = torch.empty((B, K * K, H, W), device=x1.device, dtype=torch.float32)
    else:
        _check_out("output", out, (B, K * K, H, W), x1.device)
    lib = _lib.load()
    ws, nws = _corr_workspace(lib, B, C, H, W, d, x1.device)
    _args = (x1c.data_ptr(), x2c.data_ptr(), out.data_ptr(), K * K * H * W, 0, 0.0, None,
             ws.data_ptr() if nws else None, nws, B, C, H, W, d, _lib.stream_handle(x1.device),)
    with torch.cuda.device(x1.device), _kt.timed(
        "corr_fwd", (B, C, H, W), x1.device, _kt.corr_bytes(B, C, H, W, K * K), _kt.corr_flops(B, C, H, W, K * K)
    ):
        # the _ex entry with a dense output stride: same result as usf_corr_fwd_f32,
        # plus the channel-split workspace for the small levels
        rc = lib.usf_corr_fwd_ex_f32(*_args)
    _lib.check(rc, "usf_corr_fwd_ex_f32")
    return out


def _corr_workspace(lib, B, C, H, W, d, device):
    """Caller-provided scratch for the forward's channel split (torch's caching
    allocator; empty when the shape does not split)."""
    n = int(lib.usf_corr_fwd_workspace(B, C, H, W, d))
    if n <= 0:
        return None, 0
    return torch.empty(n, device=device, dtype=torch.float32), n


def corr_backward(
    x1: torch.Tensor,
    x2: torch.Tensor,
    grad_out: torch.Tensor,
    max_displacement: int,
    need_x1: bool = True,
    need_x2: bool = True,
    gx1_out: torch.Tensor | None = None,
    gx2_out: torch.Tensor | None = None,
) -> tuple[torch.Tensor | None, torch.Tensor | None]:
    """(grad_input1, grad_input2) of :func:`corr_forward`; deterministic.

    ``gx1_out`` / ``gx2_out``: optional preallocated contiguous outputs."""
    _require_device_f32("input1", x1)
    _require_device_f32("input2", x2)
    _require_device_f32("grad_output", grad_out)
    B, C, H, W = _nchw("input1", x1)
    d = int(max_displacement)
    K = 2 * d + 1
    if tuple(grad_out.shape) != (B, K * K, H, W):
        raise ValueError(f"grad_output shape {tuple(grad_out.shape)} != {(B, K * K, H, W)}")
    if not (need_x1 or need_x2):
        return None, None
    x1c, x2c, gc = x1.contiguous(), x2.contiguous(), grad_out.contiguous()
    g1 = g2 = None
    if need_x1:
        g1 = torch.empty_like(x1c) if gx1_out is None else gx1_out
        _check_out("grad_input1", g1, (B, C, H, W), x1.device)
    if need_x2:
        g2 = torch.empty_like(x2c) if gx2_out is None else gx2_out
        _check_out("grad_input2", g2, (B, C, H, W), x1.device)
    lib = _lib.load()
    _args = (x1c.data_ptr(), x2c.data_ptr(), gc.data_ptr(), _ptr(g1), _ptr(g2), B, C, H, W, d,
             _lib.stream_handle(x1.device),)
    with torch.cuda.device(x1.device), _kt.timed(
        "corr_bwd", (B, C, H, W, need_x1, need_x2), x1.device,
        _kt.corr_bytes(B, C, H, W, K * K, True, need_x1, need_x2),
        _kt.corr_flops(B, C, H, W, K * K, True, need_x1, need_x2),
    ):
        rc = lib.usf_corr_bwd_f32(*_args)
    _lib.check(rc, "usf_corr_bwd_f32")
    return g1, g2


def _flow_view(flow: torch.Tensor, B: int, H: int, W: int) -> tuple[torch.Tensor, int]:
    """Flow tensor whose per-sample [2,H,W] block is dense, plus its batch stride.

    A channel slice such as ``flow[:, :2]`` of a contiguous [B,4,H,W] tensor
    (flow_loss.py:130-131) qualifies as-is (batch stride 4*H*W): no copy.
    """
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"flow shape {tuple(flow.shape)} != {(B, 2, H, W)}")
    s = flow.stride()
    if s[1] == H * W and s[2] == W and s[3] == 1 and (B == 1 or s[0] >= 2 * H * W):
        return flow, s[0] if B > 1 else 2 * H * W
    flow = flow.contiguous()
    return flow, 2 * H * W


def warp_forward(x: torch.Tensor, flow: torch.Tensor, pad: str = "border") -> torch.Tensor:
    """Bilinear backward warp of x by flow (warp_utils.py:97-106)."""
    _require_device_f32("x", x)
    _require_device_f32("flow12", flow)
    B, C, H, W = _nchw("x", x)
    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    if flow.device != x.device:
        raise ValueError("x and flow12 are on different devices")
    xc = x.contiguous()
    fv, fbs = _flow_view(flow, B, H, W)
    out = torch.empty_like(xc)
    lib = _lib.load()
    _args = (xc.data_ptr(), fv.data_ptr(), fbs, out.data_ptr(), B, C, H, W, PAD_MODES[pad],
             _lib.stream_handle(x.device),)
    with torch.cuda.device(x.device), _kt.timed("warp_fwd", (B, C, H, W, pad), x.device, _kt.warp_bytes(B, C, H, W)):
        rc = lib.usf_warp_fwd_f32(*_args)
    _lib.check(rc, "usf_warp_fwd_f32")
    return out


# Persistent workspaces of the *_persist_* entry points (include/unsamflow_hip.h,
# ABI 8): zeroed once when created, then left reusable by every call, so the
# per-call fill launch is gone. One per (device, op, shape). The state they
# carry (a parity word, count buffers, dirty words, an overflow buffer, the
# occlusion splat map) must see its calls in order, so each entry records the
# stream of its last eager use, and a call from another stream first makes its
# stream wait for that one (torch's wait_stream): two streams can never race a
# workspace. A HIP graph capture reuses the workspace its eager warm-up created
# (torch captures on its own stream; the capture records no fill, and replays
# are uses on the replaying stream). The cache is bounded (least recently used
# out): each warp entry holds ~88 B per pixel plus one float per element of x,
# each occlusion entry 4 B per pixel, and a training run with a changing shape
# (a partial last batch, evaluation at another resolution) must not keep every
# shape's buffers alive. A call that fails drops its entry (its state may be
# half-updated): the next call of that shape starts from a fresh zeroed buffer.
_PERSIST: "OrderedDict[tuple, list]" = OrderedDict()
PERSIST_MAX_ENTRIES = 32


def persistent_workspace(device: torch.device, op: str, shape: tuple, nbytes: int) -> torch.Tensor:
    """The zero-initialised persistent workspace of ``op`` at ``shape`` on
    ``device``, ordered after its previous use (created on first use with
    torch.zeros on the current stream, so the zeroing precedes the first call)."""
    key = (device.index, op, tuple(shape))
    cur = torch.cuda.current_stream(device)
    capturing = torch.cuda.is_current_stream_capturing()
    ent = _PERSIST.get(key)
    if ent is not None and ent[0].numel() >= nbytes:
        _PERSIST.move_to_end(key)
        if not capturing:
            if ent[1] != cur:
                cur.wait_stream(ent[1])  # the previous use on another stream comes first
            ent[1] = cur
        return ent[0]
    if capturing:
        # torch.zeros inside a capture is only recorded: the eager calls after it
        # would start from uninitialised state
        raise RuntimeError(
            f"unsamflow_amd: first use of the persistent {op} workspace for shape {tuple(shape)} inside a "
            "HIP graph capture; run the call once eagerly before capturing")
    ws = torch.zeros(nbytes, device=device, dtype=torch.uint8)
    _PERSIST[key] = [ws, cur]
    while len(_PERSIST) > PERSIST_MAX_ENTRIES:
        _PERSIST.popitem(last=False)
    return ws


def _drop_workspace(device: torch.device, op: str, shape: tuple) -> None:
    _PERSIST.pop((device.index, op, tuple(shape)), None)


def clear_persistent_workspaces() -> None:
    """Release every persistent workspace (the next call of each shape re-creates it)."""
    _PERSIST.clear()


# The largest level (H*W pixels) that takes the persistent warp backward
# (usf_warp_bwd_persist_f32); larger ones take the four-launch per-call form
# (None: every level). The library picks the persistent layout by size: up to
# 8192 pixels two launches with a dense overflow buffer, above that three (the
# overflow listed and added by the overflow pass; no zero fill). Chosen by the
# in-step time of the training step (tools/instep_ab.py, same process,
# alternating, 6 rounds; profiles/ab_r06/warp_form_list.json): KITTI L4 (64x208)
# 55.4 us in the list form vs 59.0 four-launch; the dense form there was 68.8
# (profiles/ab_r06/warp_form_instep_r2.json).
WARP_PERSIST_MAX_PIXELS: int | None = None


def warp_backward(
    x: torch.Tensor,
    flow: torch.Tensor,
    grad_out: torch.Tensor,
    pad: str = "border",
    need_x: bool = True,
    need_flow: bool = True,
) -> tuple[torch.Tensor | None, torch.Tensor | None]:
    """(grad_x, grad_flow) of :func:`warp_forward`.

    grad_x is the library's binned gather in its persistent form
    (``usf_warp_bwd_persist_f32``: one launch with LDS binning up to 512 pixels,
    two launches up to 8192, three above with the overflow pass and no zero
    fill): every source pixel is filed under its
    north-west corner cell and each target cell sums its sources in a fixed
    order, so grad_x is deterministic unless a cell receives more than 4 source
    pixels (strongly compressive flow), whose excess is added with fp32
    atomics. Its workspace (``usf_warp_bwd_persist_workspace``: ~88 B per pixel,
    plus one float per element of x up to 8192 pixels, one int per pixel above)
    is kept per (device, shape) and ordered
    across streams (:func:`persistent_workspace`). grad_flow is deterministic."""
    _require_device_f32("x", x)
    _require_device_f32("flow12", flow)
    _require_device_f32("grad_output", grad_out)
    B, C, H, W = _nchw("x", x)
    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    if tuple(grad_out.shape) != (B, C, H, W):
        raise ValueError(f"grad_output shape {tuple(grad_out.shape)} != {(B, C, H, W)}")
    if not (need_x or need_flow):
        return None, None
    xc = x.contiguous()
    fv, fbs = _flow_view(flow, B, H, W)
    gc = grad_out.contiguous()
    gx = torch.empty_like(xc) if need_x else None  # overwritten by the library
    gf = torch.empty((B, 2, H, W), device=x.device, dtype=torch.float32) if need_flow else None
    lib = _lib.load()
    # grad_x by the binned gather, persistent form (C <= 256), else the
    # four-launch form with a per-call workspace from torch's caching allocator
    # (the C ABI's limits of the persistent form: a 32-bit dirty mask of channel
    # groups, packed (y, x), both count buffers under 32-bit byte offsets)
    persist = need_x and C <= 256 and H < 32768 and W < 65536 and 8 * B * (H + 1) * (W + 1) < 2 ** 31
    if WARP_PERSIST_MAX_PIXELS is not None and H * W > WARP_PERSIST_MAX_PIXELS:
        persist = False
    with torch.cuda.device(x.device):
        if persist:
            nws = int(lib.usf_warp_bwd_persist_workspace(B, C, H, W))
            ws = persistent_workspace(x.device, "warp_bwd", (B, C, H, W), nws)
        else:
            nws = int(lib.usf_warp_bwd_workspace(B, H, W)) if need_x else 0
            ws = torch.empty(nws, device=x.device, dtype=torch.uint8) if nws > 0 else None
        fn = lib.usf_warp_bwd_persist_f32 if persist else lib.usf_warp_bwd_ex_f32
        _args = (xc.data_ptr(), fv.data_ptr(), fbs, gc.data_ptr(), _ptr(gx), _ptr(gf), _ptr(ws), nws, B, C, H, W,
                 PAD_MODES[pad], _lib.stream_handle(x.device),)
        with _kt.timed("warp_bwd", (B, C, H, W, pad, need_x, need_flow), x.device,
                       _kt.warp_bytes(B, C, H, W, True, need_x, need_flow)):
            rc = fn(*_args)
    if rc != 0 and persist:
        _drop_workspace(x.device, "warp_bwd", (B, C, H, W))
    _lib.check(rc, "usf_warp_bwd_persist_f32" if persist else "usf_warp_bwd_ex_f32")
    return gx, gf


def _flow_arg(flow: torch.Tensor, name: str) -> tuple[torch.Tensor, int, int, int, int]:
    _require_device_f32(name, flow)
    if flow.dim() != 4 or flow.shape[1] != 2:
        raise ValueError(f"{name} must be [B,2,H,W], got {tuple(flow.shape)}")
    B, _, H, W = flow.shape
    fv, fbs = _flow_view(flow, B, H, W)
    return fv, fbs, B, H, W


def splat_map(flow: torch.Tensor, absolute: bool = False) -> torch.Tensor:
    """Forward bilinear splat of unit mass (warp_utils.py:26-94) -> [B,1,H,W].

    ``absolute``: ``flow`` holds target coordinates (get_corresponding_map's
    argument) instead of displacements from the pixel grid."""
    fv, fbs, B, H, W = _flow_arg(flow, "flow")
    out = torch.empty((B, 1, H, W), device=flow.device, dtype=torch.float32)
    lib = _lib.load()
    _args = (fv.data_ptr(), fbs, out.data_ptr(), B, H, W, int(bool(absolute)), _lib.stream_handle(flow.device),)
    with torch.cuda.device(flow.device), _kt.timed("splat", (B, 1, H, W, bool(absolute)), flow.device,
                                                     4 * B * H * W * 3):
        rc = lib.usf_splat_map_f32(*_args)
    _lib.check(rc, "usf_splat_map_f32")
    return out


def occ_backward(flow21: torch.Tensor, th: float = 0.2) -> torch.Tensor:
    """Occlusion mask get_occu_mask_backward (warp_utils.py:120-126) -> [B,1,H,W] float."""
    fv, fbs, B, H, W = _flow_arg(flow21, "flow21")
    out = torch.empty((B, 1, H, W), device=flow21.device, dtype=torch.float32)
    lib = _lib.load()
    with torch.cuda.device(flow21.device):
        # the splat map lives in a persistent zeroed buffer that the threshold pass
        # re-zeroes (usf_occ_backward_persist_f32: two launches, no fill)
        nmap = 4 * B * H * W
        ws = persistent_workspace(flow21.device, "occ_bwd", (B, H, W), nmap)
        _args = (fv.data_ptr(), fbs, out.data_ptr(), ws.data_ptr(), nmap, B, H, W, float(th),
                 _lib.stream_handle(flow21.device),)
        with _kt.timed("occ_bwd", (B, 1, H, W), flow21.device, 4 * B * H * W * 3):
            rc = lib.usf_occ_backward_persist_f32(*_args)
    if rc != 0:
        _drop_workspace(flow21.device, "occ_bwd", (B, H, W))
    _lib.check(rc, "usf_occ_backward_persist_f32")
    return out


def occ_vis_pair(flow4: torch.Tensor, th: float = 0.2) -> torch.Tensor:
    """Both visibility masks of a with_bk loss at once (flow_loss.py:101-103):
    ``vis[0] = 1 - get_occu_mask_backward(flow4[:, 2:], th)``, ``vis[1] = 1 -
    get_occu_mask_backward(flow4[:, :2], th)`` -> [2,B,1,H,W] (each half a
    contiguous [B,1,H,W]): one splat launch over both flow halves into a
    persistent interleaved map and one threshold pass (usf_occ_vis_pair_persist_f32)
    instead of two splats, two thresholds and two ``1 - occ`` passes."""
    _require_device_f32("flow4", flow4)
    if flow4.dim() != 4 or flow4.shape[1] != 4:
        raise ValueError(f"flow4 must be [B,4,H,W], got {tuple(flow4.shape)}")
    f = flow4.contiguous()
    B, _, H, W = f.shape
    vis = torch.empty((2, B, 1, H, W), device=f.device, dtype=torch.float32)
    lib = _lib.load()
    with torch.cuda.device(f.device):
        nmap = 8 * B * H * W
        ws = persistent_workspace(f.device, "occ_vis_pair", (B, H, W), nmap)
        _args = (f.data_ptr(), 4 * H * W, vis.data_ptr(), ws.data_ptr(), nmap, B, H, W, float(th),
                 _lib.stream_handle(f.device),)
        with _kt.timed("occ_vis_pair", (B, 1, H, W), f.device, 4 * B * H * W * 6):
            rc = lib.usf_occ_vis_pair_persist_f32(*_args)
    if rc != 0:
        _drop_workspace(f.device, "occ_vis_pair", (B, H, W))
    _lib.check(rc, "usf_occ_vis_pair_persist_f32")
    return vis


def occ_bidirection(flow12: torch.Tensor, flow21: torch.Tensor, scale: float = 0.01, bias: float = 0.5
                    ) -> torch.Tensor:
    """Occlusion mask get_occu_mask_bidirection (warp_utils.py:109-117) -> [B,1,H,W] float, one kernel."""
    f1, bs1, B, H, W = _flow_arg(flow12, "flow12")
    f2, bs2, B2, H2, W2 = _flow_arg(flow21, "flow21")
    if (B2, H2, W2) != (B, H, W):
        raise ValueError(f"flow21 shape {tuple(flow21.shape)} != flow12 shape {tuple(flow12.shape)}")
    out = torch.empty((B, 1, H, W), device=flow12.device, dtype=torch.float32)
    lib = _lib.load()
    _args = (f1.data_ptr(), bs1, f2.data_ptr(), bs2, out.data_ptr(), B, H, W, float(scale), float(bias),
             _lib.stream_handle(flow12.device),)
    with torch.cuda.device(flow12.device), _kt.timed("occ_bidir", (B, 1, H, W), flow12.device,
                                                       4 * B * H * W * 5):
        rc = lib.usf_occ_bidirection_f32(*_args)
    _lib.check(rc, "usf_occ_bidirection_f32")
    return out


def _photo_args(src, tgt, mask, flow):
    for n, t in (("src", src), ("tgt", tgt), ("mask", mask)):
        _require_device_f32(n, t)
    B, C, H, W = _nchw("src", src)
    if tuple(tgt.shape) != (B, C, H, W) or tuple(mask.shape) != (B, 1, H, W):
        raise ValueError(f"tgt {tuple(tgt.shape)} / mask {tuple(mask.shape)} do not match src {(B, C, H, W)}")
    if C > 3:
        raise NotImplementedError(f"fused photometric loss supports C <= 3 image channels, got {C}")
    if flow is None:
        return src.contiguous(), tgt.contiguous(), mask.contiguous(), B, C, H, W
    _require_device_f32("flow", flow)
    fv, fbs = _flow_view(flow, B, H, W)
    return src.contiguous(), tgt.contiguous(), mask.contiguous(), fv, fbs, B, C, H, W


def photo_loss_forward(src, tgt, mask, flow, pad: str = "border", w_l1: float = 0.15, w_ssim: float = 0.85,
                       need_grad: bool = False):
    """Fused warp + occlusion-aware L1/SSIM photometric loss of one scale and
    direction (flow_loss.py:127-148, loss_blocks.py:53-72) -> (out, basis):
    ``out`` = tensor [3] on the device {loss, c_l1, c_ssim}; with ``need_grad``
    ``basis`` = [B,4,H,W], the per-pixel flow-gradient basis computed in the
    same pass (dL/dflow = c_l1 * basis[:, :2] + c_ssim * basis[:, 2:]), else None."""
    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    s, t, m, fv, fbs, B, C, H, W = _photo_args(src, tgt, mask, flow)
    lib = _lib.load()
    partials = torch.empty(lib.usf_photo_loss_partials(B, H, W), device=src.device, dtype=torch.float32)
    out = torch.empty(3, device=src.device, dtype=torch.float32)
    basis = torch.empty((B, 4, H, W), device=src.device, dtype=torch.float32) if need_grad else None
    # algorithmic bytes: src, tgt, mask, flow read once; the basis written once
    nbytes = 4 * B * H * W * (2 * C + 3 + (4 if need_grad else 0))
    op = "photo_fwd_grad" if need_grad else "photo_fwd"
    _args = (s.data_ptr(), t.data_ptr(), m.data_ptr(), fv.data_ptr(), fbs, partials.data_ptr(), out.data_ptr(),
             basis.data_ptr() if need_grad else None, B, C, H, W, PAD_MODES[pad], float(w_l1), float(w_ssim),
             _lib.stream_handle(src.device),)
    with torch.cuda.device(src.device), _kt.timed(op, (B, C, H, W, pad), src.device, nbytes):
        rc = lib.usf_photo_loss_fwd_f32(*_args)
    _lib.check(rc, "usf_photo_loss_fwd_f32")
    return out, basis


def photo_loss_pair_forward(flow, im1, im2, mask1, mask2, pad: str = "border", w_l1: float = 0.15,
                            w_ssim: float = 0.85, need_grad: bool = False):
    """Both directions of a with_bk scale in one launch (flow_loss.py:130-131):
    direction 0 = loss(im1, warp(im2, flow[:, :2]), mask1), direction 1 =
    loss(im2, warp(im1, flow[:, 2:]), mask2) -> (out [6] = {loss, c_l1, c_ssim}
    per direction, basis [B,8,H,W] (= [B,2,4,H,W]) or None)."""
    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    a, b_, m1, B, C, H, W = _photo_args(im1, im2, mask1, None)
    m2 = mask2.contiguous()
    _require_device_f32("mask2", m2)
    if tuple(m2.shape) != (B, 1, H, W):
        raise ValueError(f"mask2 {tuple(m2.shape)} does not match {(B, 1, H, W)}")
    _require_device_f32("flow", flow)
    if tuple(flow.shape) != (B, 4, H, W):
        raise ValueError(f"flow must be [B,4,H,W] = {(B, 4, H, W)}, got {tuple(flow.shape)}")
    fv = flow if flow[0].is_contiguous() else flow.contiguous()
    fbs = fv.stride(0) if B > 1 else 4 * H * W
    lib = _lib.load()
    partials = torch.empty(2 * lib.usf_photo_loss_partials(B, H, W), device=im1.device, dtype=torch.float32)
    out = torch.empty(6, device=im1.device, dtype=torch.float32)
    basis = torch.empty((B, 8, H, W), device=im1.device, dtype=torch.float32) if need_grad else None
    # algorithmic bytes (each input read once): im1 and im2 (2C), the
    # 4-channel flow, both masks; with the gradient the 8 basis planes written once
    nbytes = 4 * B * H * W * (2 * C + 4 + 2 + (8 if need_grad else 0))
    op = "photo_pair_grad" if need_grad else "photo_pair"
    _args = (a.data_ptr(), b_.data_ptr(), m1.data_ptr(), m2.data_ptr(), fv.data_ptr(), fbs, partials.data_ptr(),
             out.data_ptr(), basis.data_ptr() if need_grad else None, B, C, H, W, PAD_MODES[pad], float(w_l1),
             float(w_ssim), _lib.stream_handle(im1.device),)
    with torch.cuda.device(im1.device), _kt.timed(op, (B, C, H, W, pad), im1.device, nbytes):
        rc = lib.usf_photo_loss_pair_fwd_f32(*_args)
    _lib.check(rc, "usf_photo_loss_pair_fwd_f32")
    return out, basis


def _host_array(ctype, values):
    return (ctype * len(values))(*values)


def photo_loss_pyramid_forward(flows, im1s, im2s, masks1, masks2, pad: str = "border", w_l1: float = 0.15,
                               w_ssim: float = 0.85, need_grad: bool = False):
    """:func:`photo_loss_pair_forward` for up to 4 loss scales in one launch
    (usf_photo_loss_pyramid_fwd_f32; the largest scale first) -> (out
    [nscale, 6] = {loss, c_l1, c_ssim} per direction per scale, bases: a list
    of [B,8,H_k,W_k] or None)."""
    import ctypes

    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    n = len(flows)
    if not 1 <= n <= 4 or not (len(im1s) == len(im2s) == len(masks1) == len(masks2) == n):
        raise ValueError(f"1..4 scales with one flow, two images and two masks each (got {n})")
    args = []
    for f, a, b_, m1, m2 in zip(flows, im1s, im2s, masks1, masks2):
        a, b_, m1, B, C, H, W = _photo_args(a, b_, m1, None)
        m2 = m2.contiguous()
        _require_device_f32("mask2", m2)
        _require_device_f32("flow", f)
        if tuple(m2.shape) != (B, 1, H, W) or tuple(f.shape) != (B, 4, H, W):
            raise ValueError(f"scale {len(args)}: mask2 {tuple(m2.shape)} / flow {tuple(f.shape)} vs {(B, C, H, W)}")
        fv = f if f[0].is_contiguous() else f.contiguous()
        args.append((fv, a, b_, m1, m2, B, C, H, W, fv.stride(0) if B > 1 else 4 * H * W))
    B, C = args[0][5], args[0][6]
    if any(x[5] != B or x[6] != C for x in args):
        raise ValueError("every scale needs the same batch and channel count")
    dev = args[0][1].device
    Hs = _host_array(ctypes.c_int, [x[7] for x in args])
    Ws = _host_array(ctypes.c_int, [x[8] for x in args])
    lib = _lib.load()
    npart = int(lib.usf_photo_loss_pyramid_partials(n, Hs, Ws, B))
    partials = torch.empty(npart, device=dev, dtype=torch.float32)
    out = torch.empty((n, 6), device=dev, dtype=torch.float32)
    bases = [torch.empty((B, 8, x[7], x[8]), device=dev, dtype=torch.float32) for x in args] if need_grad else None
    ptrs = lambda i: _host_array(ctypes.c_void_p, [x[i].data_ptr() for x in args])  # noqa: E731
    nbytes = sum(4 * B * x[7] * x[8] * (2 * C + 4 + 2 + (8 if need_grad else 0)) for x in args)
    op = "photo_pyr_grad" if need_grad else "photo_pyr"
    key = (B, C) + tuple(v for x in args for v in (x[7], x[8])) + (pad,)
    _args = (n, ptrs(1), ptrs(2), ptrs(3), ptrs(4), ptrs(0), _host_array(ctypes.c_longlong, [x[9] for x in args]),
             Hs, Ws, partials.data_ptr(), npart, out.data_ptr(),
             _host_array(ctypes.c_void_p, [t.data_ptr() for t in bases]) if need_grad else None, B, C,
             PAD_MODES[pad], float(w_l1), float(w_ssim), _lib.stream_handle(dev),)
    with torch.cuda.device(dev), _kt.timed(op, key, dev, nbytes):
        rc = lib.usf_photo_loss_pyramid_fwd_f32(*_args)
    _lib.check(rc, "usf_photo_loss_pyramid_fwd_f32")
    return out, bases


def photo_loss_pyramid_backward(bases, coef, grad_losses):
    """d(loss)/d(flow_k) * grad for every scale of :func:`photo_loss_pyramid_forward`
    in one launch: bases [B,8,H_k,W_k], coef = its out [nscale, 6], grad_losses
    [nscale, 2] -> list of [B,4,H_k,W_k] (deterministic)."""
    import ctypes

    n = len(bases)
    for t in bases:
        _require_device_f32("basis", t)
    B = bases[0].shape[0]
    dev = bases[0].device
    gl = grad_losses.reshape(-1).to(torch.float32).contiguous()
    if gl.numel() != 2 * n or coef.numel() != 6 * n:
        raise ValueError(f"grad_losses / coef sizes {gl.numel()} / {coef.numel()} for {n} scales")
    gflows = [torch.empty((B, 4) + tuple(t.shape[2:]), device=dev, dtype=torch.float32) for t in bases]
    Hs = _host_array(ctypes.c_int, [t.shape[2] for t in bases])
    Ws = _host_array(ctypes.c_int, [t.shape[3] for t in bases])
    lib = _lib.load()
    key = (B, 2) + tuple(v for t in bases for v in t.shape[2:])
    nbytes = sum(4 * B * t.shape[2] * t.shape[3] * 12 for t in bases)
    _args = (n, _host_array(ctypes.c_void_p, [t.contiguous().data_ptr() for t in bases]),
             coef.contiguous().data_ptr(), gl.data_ptr(),
             _host_array(ctypes.c_void_p, [t.data_ptr() for t in gflows]), Hs, Ws, B, _lib.stream_handle(dev),)
    with torch.cuda.device(dev), _kt.timed("photo_pyr_bwd", key, dev, nbytes):
        rc = lib.usf_photo_loss_pyramid_bwd_f32(*_args)
    _lib.check(rc, "usf_photo_loss_pyramid_bwd_f32")
    return gflows


def photo_loss_backward(basis, coef, grad_loss):
    """d(photo loss)/d(flow) * grad_loss from the forward's gradient basis
    ([B,4,H,W] one direction, [B,8,H,W] a pair) and coefficients ->
    [B,2,H,W] / [B,4,H,W] (deterministic)."""
    _require_device_f32("basis", basis)
    B, K, H, W = _nchw("basis", basis)
    if K not in (4, 8):
        raise ValueError(f"gradient basis must be [B,4,H,W] or [B,8,H,W], got {tuple(basis.shape)}")
    ndir = K // 4
    basis = basis.contiguous()
    gl = grad_loss.reshape(-1).to(torch.float32).contiguous()
    if gl.numel() != ndir:
        raise ValueError(f"grad_loss has {gl.numel()} elements for {ndir} direction(s)")
    gflow = torch.empty((B, 2 * ndir, H, W), device=basis.device, dtype=torch.float32)
    lib = _lib.load()
    _args = (basis.data_ptr(), coef.data_ptr(), gl.data_ptr(), gflow.data_ptr(), B, H, W, ndir,
             _lib.stream_handle(basis.device),)
    with torch.cuda.device(basis.device), _kt.timed("photo_bwd", (B, ndir, H, W), basis.device,
                                                      4 * B * H * W * 6 * ndir):
        rc = lib.usf_photo_loss_bwd_f32(*_args)
    _lib.check(rc, "usf_photo_loss_bwd_f32")
    return gflow


def _plane_slice_stride(name: str, t: torch.Tensor, shape) -> int:
    """Batch stride of a [B,K,H,W] channel slice whose per-sample planes are dense."""
    B, K, H, W = shape
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} shape {tuple(t.shape)} != {tuple(shape)}")
    s = t.stride()
    if s[1] != H * W or s[2] != W or s[3] != 1 or (B > 1 and s[0] < K * H * W):
        raise ValueError(f"{name} must be a channel slice of an NCHW-contiguous tensor (strides {s})")
    return s[0] if B > 1 else K * H * W


def corr_act_mask(B: int, H: int, W: int, max_displacement: int, device, C: int | None = None
                  ) -> torch.Tensor | None:
    """An empty LeakyReLU sign mask for :func:`corr_forward_ex` (int64 words,
    [B,2d+1,H,ceil(W/4)]), at every level: the unsplit forward writes it in its
    epilogue, the channel-split forward of the small levels in its reduce.
    ``C`` is accepted for call-site compatibility (the mask no longer depends
    on it)."""
    lib = _lib.load()
    n = int(lib.usf_corr_act_mask_words(B, H, W, int(max_displacement)))
    if n == 0:
        return None
    return torch.empty((B, 2 * int(max_displacement) + 1, H, (W + 3) // 4), device=device, dtype=torch.int64)


def corr_forward_ex(x1: torch.Tensor, x2: torch.Tensor, max_displacement: int, out: torch.Tensor,
                    leaky_slope: float | None = None, act_mask: torch.Tensor | None = None) -> torch.Tensor:
    """:func:`corr_forward` into ``out``, a [B,(2d+1)^2,H,W] channel slice of a
    larger NCHW buffer (the flow estimator's concat input), with the decoder's
    LeakyReLU applied in the kernel epilogue when ``leaky_slope`` is given; with
    ``act_mask`` (:func:`corr_act_mask`) the epilogue also writes the output's
    sign bits for :func:`corr_backward_ex`."""
    _require_device_f32("input1", x1)
    _require_device_f32("input2", x2)
    _require_device_f32("output", out)
    B, C, H, W = _nchw("input1", x1)
    if x2.shape != x1.shape:
        raise ValueError(f"input2 shape {tuple(x2.shape)} != input1 shape {tuple(x1.shape)}")
    d = int(max_displacement)
    K = 2 * d + 1
    obs = _plane_slice_stride("output", out, (B, K * K, H, W))
    x1c, x2c = x1.contiguous(), x2.contiguous()
    lib = _lib.load()
    act = 0 if leaky_slope is None else 1
    if act_mask is not None:
        if act == 0 or act_mask.dtype != torch.int64 or not act_mask.is_contiguous() \
                or act_mask.numel() != int(lib.usf_corr_act_mask_words(B, H, W, d)):
            raise ValueError("act_mask: a contiguous int64 corr_act_mask() tensor with leaky_slope set")
    ws, nws = _corr_workspace(lib, B, C, H, W, d, x1.device)
    # the decoder's site (LeakyReLU epilogue into the concat slice, + the sign mask)
    # is its own timing site, so its device time is measured on the same call
    op = "corr_fwd_leaky" if act else "corr_fwd"
    nbytes = _kt.corr_bytes(B, C, H, W, K * K) + (8 * act_mask.numel() if act_mask is not None else 0)
    _args = (x1c.data_ptr(), x2c.data_ptr(), out.data_ptr(), obs, act, float(leaky_slope or 0.0), _ptr(act_mask),
             ws.data_ptr() if nws else None, nws, B, C, H, W, d, _lib.stream_handle(x1.device),)
    with torch.cuda.device(x1.device), _kt.timed(
        op, (B, C, H, W), x1.device, nbytes, _kt.corr_flops(B, C, H, W, K * K)
    ):
        rc = lib.usf_corr_fwd_ex_f32(*_args)
    _lib.check(rc, "usf_corr_fwd_ex_f32")
    return out


def corr_backward_ex(x1: torch.Tensor, x2: torch.Tensor, grad_out: torch.Tensor, max_displacement: int,
                     need_x1: bool = True, need_x2: bool = True, act_out: torch.Tensor | None = None,
                     leaky_slope: float = 0.1, act_mask: torch.Tensor | None = None,
                     ) -> tuple[torch.Tensor | None, torch.Tensor | None]:
    """:func:`corr_backward` reading ``grad_out`` as a channel slice of the concat
    gradient; with ``act_out`` (the forward's activated slice) the LeakyReLU
    derivative is applied first (one dense pass into a scratch); with
    ``act_mask`` (the forward's sign mask) it is applied inside the backward
    kernel's gradient loads instead, and ``act_out`` is not read."""
    _require_device_f32("input1", x1)
    _require_device_f32("input2", x2)
    _require_device_f32("grad_output", grad_out)
    B, C, H, W = _nchw("input1", x1)
    d = int(max_displacement)
    K = 2 * d + 1
    gbs = _plane_slice_stride("grad_output", grad_out, (B, K * K, H, W))
    scratch = None
    lib = _lib.load()
    if act_mask is not None:
        if act_mask.dtype != torch.int64 or not act_mask.is_contiguous() \
                or act_mask.numel() != int(lib.usf_corr_act_mask_words(B, H, W, d)):
            raise ValueError("act_mask: the forward's contiguous int64 corr_act_mask() tensor")
        act_out = None
    elif act_out is not None:
        _require_device_f32("act_out", act_out)
        if _plane_slice_stride("act_out", act_out, (B, K * K, H, W)) != gbs:
            raise ValueError("act_out and grad_output must share the batch stride")
        n = int(lib.usf_corr_bwd_ex_scratch(B, C, H, W, d))
        if n:
            scratch = torch.empty(n, device=x1.device, dtype=torch.float32)
    if not (need_x1 or need_x2):
        return None, None
    x1c, x2c = x1.contiguous(), x2.contiguous()
    g1 = torch.empty_like(x1c) if need_x1 else None
    g2 = torch.empty_like(x2c) if need_x2 else None
    # with the LeakyReLU derivative the site also reads the activated output
    # once (what leaky_relu_backward needs): a distinct site, its bytes included
    # (with the sign mask instead: its words are the derivative's input)
    op = "corr_bwd" if act_out is None and act_mask is None else "corr_bwd_leaky"
    nbytes = _kt.corr_bytes(B, C, H, W, K * K, True, need_x1, need_x2)
    if act_out is not None:
        nbytes += 4 * B * H * W * K * K
    elif act_mask is not None:
        nbytes += 8 * act_mask.numel()
    _args = (x1c.data_ptr(), x2c.data_ptr(), grad_out.data_ptr(), gbs, _ptr(act_out), _ptr(act_mask),
             float(leaky_slope), _ptr(scratch), _ptr(g1), _ptr(g2), B, C, H, W, d, _lib.stream_handle(x1.device),)
    with torch.cuda.device(x1.device), _kt.timed(
        op, (B, C, H, W, need_x1, need_x2), x1.device, nbytes,
        _kt.corr_flops(B, C, H, W, K * K, True, need_x1, need_x2),
    ):
        rc = lib.usf_corr_bwd_ex_f32(*_args)
    _lib.check(rc, "usf_corr_bwd_ex_f32")
    return g1, g2


def flow_upsample(flow: torch.Tensor, factor: int) -> torch.Tensor:
    """F.interpolate(flow * factor, scale_factor=factor, mode="bilinear", align_corners=True)."""
    _require_device_f32("flow", flow)
    B, C, H, W = _nchw("flow", flow)
    k = int(factor)
    fc = flow.contiguous()
    out = torch.empty((B, C, H * k, W * k), device=flow.device, dtype=torch.float32)
    lib = _lib.load()
    _args = (fc.data_ptr(), out.data_ptr(), B, C, H, W, k, _lib.stream_handle(flow.device),)
    with torch.cuda.device(flow.device), _kt.timed("upsample", (B, C, H, W, k), flow.device,
                                                     4 * B * C * H * W * (1 + k * k)):
        rc = lib.usf_flow_upsample_f32(*_args)
    _lib.check(rc, "usf_flow_upsample_f32")
    return out


def warp_forward_up(x: torch.Tensor, coarse_flow: torch.Tensor, pad: str = "border") -> tuple[torch.Tensor, torch.Tensor]:
    """(up, out): up = F.interpolate(coarse_flow * 2, scale_factor=2, bilinear,
    align_corners=True) and out = flow_warp(x, up) (pwclite.py:299-302) in ONE
    launch (``usf_warp_fwd_up_f32``); the same numbers as :func:`flow_upsample`
    followed by :func:`warp_forward`."""
    _require_device_f32("x", x)
    _require_device_f32("coarse_flow", coarse_flow)
    B, C, H, W = _nchw("x", x)
    if pad not in PAD_MODES:
        raise NotImplementedError(f"flow_warp padding mode {pad!r} (supported: border, zeros)")
    if tuple(coarse_flow.shape) != (B, 2, H // 2, W // 2) or H % 2 or W % 2:
        raise ValueError(f"coarse flow shape {tuple(coarse_flow.shape)} is not [B,2,H/2,W/2] of x {(B, C, H, W)}")
    xc, fc = x.contiguous(), coarse_flow.contiguous()
    up = torch.empty((B, 2, H, W), device=x.device, dtype=torch.float32)
    out = torch.empty_like(xc)
    lib = _lib.load()
    _args = (xc.data_ptr(), fc.data_ptr(), up.data_ptr(), out.data_ptr(), B, C, H, W, PAD_MODES[pad],
             _lib.stream_handle(x.device),)
    with torch.cuda.device(x.device), _kt.timed("warp_fwd_up", (B, C, H, W, pad), x.device,
                                                  _kt.warp_bytes(B, C, H, W) + 4 * B * 2 * (H // 2) * (W // 2)):
        rc = lib.usf_warp_fwd_up_f32(*_args)
    _lib.check(rc, "usf_warp_fwd_up_f32")
    return up, out


def flow_upsample_backward(grad_out: torch.Tensor, factor: int, grad_out2: torch.Tensor | None = None) -> torch.Tensor:
    """Backward of :func:`flow_upsample` for grad_out (+ grad_out2, summed per
    element inside the kernel: ``usf_flow_upsample_bwd_sum_f32``)."""
    _require_device_f32("grad_out", grad_out)
    B, C, Ho, Wo = _nchw("grad_out", grad_out)
    k = int(factor)
    if Ho % k or Wo % k:
        raise ValueError(f"grad_out spatial size {(Ho, Wo)} is not a multiple of {k}")
    H, W = Ho // k, Wo // k
    gc = grad_out.contiguous()
    gx = torch.empty((B, C, H, W), device=grad_out.device, dtype=torch.float32)
    lib = _lib.load()
    if grad_out2 is not None:
        _require_device_f32("grad_out2", grad_out2)
        if grad_out2.shape != grad_out.shape:
            raise ValueError(f"grad_out2 shape {tuple(grad_out2.shape)} != {tuple(grad_out.shape)}")
        g2 = grad_out2.contiguous()
        _args = (gc.data_ptr(), g2.data_ptr(), gx.data_ptr(), B, C, H, W, k, _lib.stream_handle(grad_out.device),)
        with torch.cuda.device(grad_out.device), _kt.timed("upsample_bwd", (B, C, H, W, k), grad_out.device,
                                                             4 * B * C * H * W * (1 + 2 * k * k)):
            rc = lib.usf_flow_upsample_bwd_sum_f32(*_args)
        _lib.check(rc, "usf_flow_upsample_bwd_sum_f32")
        return gx
    _args = (gc.data_ptr(), gx.data_ptr(), B, C, H, W, k, _lib.stream_handle(grad_out.device),)
    with torch.cuda.device(grad_out.device), _kt.timed("upsample_bwd", (B, C, H, W, k), grad_out.device,
                                                         4 * B * C * H * W * (1 + k * k)):
        rc = lib.usf_flow_upsample_bwd_f32(*_args)
    _lib.check(rc, "usf_flow_upsample_bwd_f32")
    return gx


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor, factor: int = 4,
                    mask_scale: float = 0.25) -> torch.Tensor:
    """UpFlowNetwork.upsample_flow(flow, mask_scale * mask) (pwclite.py:148-166):
    flow [B,2,H,W], mask [B,9*f*f,H,W] (the convs' raw output) -> [B,2,fH,fW]."""
    _require_device_f32("flow", flow)
    _require_device_f32("mask", mask)
    B, C, H, W = _nchw("flow", flow)
    f = int(factor)
    if C != 2 or tuple(mask.shape) != (B, 9 * f * f, H, W):
        raise ValueError(f"convex_upsample: flow {tuple(flow.shape)} / mask {tuple(mask.shape)} (want [B,2,H,W] / "
                         f"[B,{9 * f * f},H,W])")
    fc, mc = flow.contiguous(), mask.contiguous()
    out = torch.empty((B, 2, f * H, f * W), device=flow.device, dtype=torch.float32)
    lib = _lib.load()
    nbytes = 4 * B * H * W * (2 + 11 * f * f)
    _args = (fc.data_ptr(), mc.data_ptr(), out.data_ptr(), B, H, W, f, float(mask_scale),
             _lib.stream_handle(flow.device),)
    with torch.cuda.device(flow.device), _kt.timed("convex_up", (B, H, W, f), flow.device, nbytes):
        rc = lib.usf_convex_upsample_f32(*_args)
    _lib.check(rc, "usf_convex_upsample_f32")
    return out


def convex_upsample_backward(flow: torch.Tensor, mask: torch.Tensor, grad_out: torch.Tensor, factor: int = 4,
                             mask_scale: float = 0.25, need_flow: bool = True, need_mask: bool = True):
    """(grad_flow, grad_mask) of convex_upsample; grad_mask is w.r.t. the raw mask."""
    _require_device_f32("grad_out", grad_out)
    B, _, H, W = _nchw("flow", flow)
    f = int(factor)
    if tuple(grad_out.shape) != (B, 2, f * H, f * W):
        raise ValueError(f"convex_upsample_backward: grad_out {tuple(grad_out.shape)}")
    if not (need_flow or need_mask):
        return None, None
    fc, mc, gc = flow.contiguous(), mask.contiguous(), grad_out.contiguous()
    gf = torch.empty((B, 2, H, W), device=flow.device, dtype=torch.float32) if need_flow else None
    gm = torch.empty_like(mc) if need_mask else None
    lib = _lib.load()
    scratch = None
    if need_flow:
        scratch = torch.empty(int(lib.usf_convex_upsample_bwd_scratch(B, H, W)), device=flow.device,
                              dtype=torch.float32)
    nbytes = 4 * B * H * W * (2 + 9 * f * f + 2 * f * f + (2 if need_flow else 0) + (9 * f * f if need_mask else 0))
    _args = (fc.data_ptr(), mc.data_ptr(), gc.data_ptr(), _ptr(gf), _ptr(gm), _ptr(scratch), B, H, W, f,
             float(mask_scale), _lib.stream_handle(flow.device),)
    with torch.cuda.device(flow.device), _kt.timed("convex_up_bwd", (B, H, W, f), flow.device, nbytes):
        rc = lib.usf_convex_upsample_bwd_f32(*_args)
    _lib.check(rc, "usf_convex_upsample_bwd_f32")
    return gf, gm


def _level_sizes(flows):
    import ctypes

    return (_host_array(ctypes.c_int, [f.shape[2] for f in flows]),
            _host_array(ctypes.c_int, [f.shape[3] for f in flows]))


def convex_upsample_pyramid(flows, masks, factor: int = 4, mask_scale: float = 0.25):
    """:func:`convex_upsample` of every decoder level in one launch
    (usf_convex_upsample_pyramid_f32): flows [B,2,H_l,W_l], masks
    [B,9f^2,H_l,W_l] -> list of [B,2,fH_l,fW_l]; the same numbers as the
    per-level calls."""
    import ctypes

    n = len(flows)
    fl = [f.contiguous() for f in flows]
    mk = [m.contiguous() for m in masks]
    for f, m in zip(fl, mk):
        _require_device_f32("flow", f)
        _require_device_f32("mask", m)
    B, f_ = fl[0].shape[0], int(factor)
    outs = [torch.empty((B, 2, f_ * f.shape[2], f_ * f.shape[3]), device=f.device, dtype=torch.float32) for f in fl]
    Hs, Ws = _level_sizes(fl)
    lib = _lib.load()
    dev = fl[0].device
    key = (B,) + tuple(v for f in fl for v in f.shape[2:]) + (f_,)
    nbytes = sum(4 * B * f.shape[2] * f.shape[3] * (2 + 11 * f_ * f_) for f in fl)
    ptrs = lambda ts: _host_array(ctypes.c_void_p, [t.data_ptr() for t in ts])  # noqa: E731
    _args = (n, ptrs(fl), ptrs(mk), ptrs(outs), Hs, Ws, B, f_, float(mask_scale), _lib.stream_handle(dev),)
    with torch.cuda.device(dev), _kt.timed("convex_pyr", key, dev, nbytes):
        rc = lib.usf_convex_upsample_pyramid_f32(*_args)
    _lib.check(rc, "usf_convex_upsample_pyramid_f32")
    return outs


def convex_upsample_pyramid_backward(flows, masks, grad_outs, factor: int = 4, mask_scale: float = 0.25,
                                     need_flow: bool = True, need_mask: bool = True):
    """(grad_flows, grad_masks) lists of :func:`convex_upsample_pyramid` (None where not needed)."""
    import ctypes

    n = len(flows)
    fl = [f.contiguous() for f in flows]
    mk = [m.contiguous() for m in masks]
    go = [g.contiguous() for g in grad_outs]
    B, f_ = fl[0].shape[0], int(factor)
    if not (need_flow or need_mask):
        return None, None
    dev = fl[0].device
    gfs = [torch.empty((B, 2) + tuple(f.shape[2:]), device=dev, dtype=torch.float32) for f in fl] if need_flow else None
    gms = [torch.empty_like(m) for m in mk] if need_mask else None
    Hs, Ws = _level_sizes(fl)
    lib = _lib.load()
    nscr = int(lib.usf_convex_upsample_pyramid_bwd_scratch(n, Hs, Ws, B)) if need_flow else 0
    scratch = torch.empty(max(nscr, 1), device=dev, dtype=torch.float32)
    ptrs = lambda ts: _host_array(ctypes.c_void_p, [t.data_ptr() for t in ts])  # noqa: E731
    key = (B,) + tuple(v for f in fl for v in f.shape[2:]) + (f_,)
    ff = f_ * f_
    nbytes = sum(4 * B * f.shape[2] * f.shape[3] * (2 + 9 * ff + 2 * ff + (2 if need_flow else 0)
                                                    + (9 * ff if need_mask else 0)) for f in fl)
    _args = (n, ptrs(fl), ptrs(mk), ptrs(go), ptrs(gfs) if need_flow else None, ptrs(gms) if need_mask else None,
             scratch.data_ptr(), nscr, Hs, Ws, B, f_, float(mask_scale), _lib.stream_handle(dev),)
    with torch.cuda.device(dev), _kt.timed("convex_pyr_bwd", key, dev, nbytes):
        rc = lib.usf_convex_upsample_pyramid_bwd_f32(*_args)
    _lib.check(rc, "usf_convex_upsample_pyramid_bwd_f32")
    return gfs, gms


def area_pyramid(x: torch.Tensor):
    """The loss's image pyramid: ``[F.interpolate(x, (H >> s, W >> s), mode="area")
    for s in 1, 2, 3]`` (flow_loss.py:128-129), one read of x, bit-exact with
    torch's CPU kernel. x: [B,C,H,W] fp32 on the device, H and W multiples of 8."""
    _require_device_f32("x", x)
    B, C, H, W = _nchw("x", x)
    if H % 8 or W % 8:
        raise ValueError(f"area_pyramid needs H, W multiples of 8, got {H}x{W}")
    xc = x.contiguous()
    outs = [torch.empty((B, C, H >> s, W >> s), device=x.device, dtype=torch.float32) for s in (1, 2, 3)]
    lib = _lib.load()
    nbytes = 4 * B * C * H * W * (1 + 1 / 4 + 1 / 16 + 1 / 64)
    _args = (xc.data_ptr(), outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), B, C, H, W,
             _lib.stream_handle(x.device),)
    with torch.cuda.device(x.device), _kt.timed("area_pyramid", (B, C, H, W), x.device, int(nbytes)):
        rc = lib.usf_area_pyramid_f32(*_args)
    _lib.check(rc, "usf_area_pyramid_f32")
    return outs
