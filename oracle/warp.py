"""TEST INFRASTRUCTURE ONLY — flow_warp oracle (see oracle/__init__.py).

Restates ``utils/warp_utils.py:97-106`` in float32 numpy:

* pixel grid + flow (mesh_grid :7-13, ``base_grid + flow12`` :102),
* norm_grid (:16-23): ``g = 2.0 * v / (W - 1) - 1.0``,
* ``grid_sample(x, g, mode='bilinear', padding_mode=pad, align_corners=True)``
  (:103-105). The sampler is third-party ATen (torch 2.10.0,
  aten/src/ATen/native/cpu/GridSamplerKernel.cpp, ``ApplyGridSample`` for
  bilinear): unnormalise ``(g + 1) * ((W-1)/2)``, border clip
  ``min(W-1, max(ix, 0))`` whose gradient is 0 when ``ix <= 0`` or
  ``ix >= W-1``, weights from ``floor``; forward
  ``nw*v_nw + ne*v_ne + sw*v_sw + se*v_se``; coordinate gradient
  ``((v_ne-v_nw)*s + (v_se-v_sw)*n)*g`` / ``((v_sw-v_nw)*e + (v_se-v_ne)*w)*g``
  accumulated over channels, times the unnormalise/clip factor; input gradient
  scattered to the 4 corners.
* autograd of norm_grid back to the flow: ``du = (dgx / (W-1)) * 2``.

Parity of this restatement with the reference (CPU torch) is pinned by the
golden vectors in tests/golden (warp is "parity unpinned by the reference's own
tests" — the reference has none — and pinned only by those captures).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def _taps(flow: np.ndarray, H: int, W: int, pad: str):
    f = flow.astype(f32)
    xs = np.arange(W, dtype=f32)[None, None, :]
    ys = np.arange(H, dtype=f32)[None, :, None]
    gx = (f32(2.0) * (xs + f[:, 0])) / f32(W - 1) - f32(1.0)
    gy = (f32(2.0) * (ys + f[:, 1])) / f32(H - 1) - f32(1.0)
    sx, sy = f32(W - 1) / f32(2), f32(H - 1) / f32(2)
    ix = (gx + f32(1)) * sx
    iy = (gy + f32(1)) * sy
    mx = np.full_like(ix, sx)
    my = np.full_like(iy, sy)
    if pad == "border":
        mx = np.where((ix > 0) & (ix < f32(W - 1)), mx, f32(0))
        my = np.where((iy > 0) & (iy < f32(H - 1)), my, f32(0))
        ix = np.minimum(f32(W - 1), np.maximum(ix, f32(0)))
        iy = np.minimum(f32(H - 1), np.maximum(iy, f32(0)))
    elif pad != "zeros":
        raise NotImplementedError(pad)
    x_w = np.floor(ix)
    y_n = np.floor(iy)
    w = ix - x_w
    e = f32(1) - w
    n = iy - y_n
    s = f32(1) - n
    xw = x_w.astype(np.int64)
    yn = y_n.astype(np.int64)
    return dict(xw=xw, yn=yn, w=w, e=e, n=n, s=s, mx=mx, my=my)


def _corners(t, H, W):
    xw, yn = t["xw"], t["yn"]
    out = []
    for cx, cy in ((xw, yn), (xw + 1, yn), (xw, yn + 1), (xw + 1, yn + 1)):  # nw, ne, sw, se
        m = (cx >= 0) & (cx < W) & (cy >= 0) & (cy < H)
        out.append((np.clip(cx, 0, W - 1), np.clip(cy, 0, H - 1), m))
    return out


def _gather(x, cx, cy, m):
    B = x.shape[0]
    bi = np.arange(B)[:, None, None]
    v = x[bi, :, cy, cx]  # [B,H,W,C]
    v = np.moveaxis(v, -1, 1)
    return np.where(m[:, None], v, f32(0))


def warp_forward_np(x: np.ndarray, flow: np.ndarray, pad: str = "border") -> np.ndarray:
    x = x.astype(f32)
    B, C, H, W = x.shape
    t = _taps(flow, H, W, pad)
    (cnw, cne, csw, cse) = _corners(t, H, W)
    s, n, w, e = (t[k][:, None] for k in "snwe")
    v_nw, v_ne, v_sw, v_se = (_gather(x, *c) for c in (cnw, cne, csw, cse))
    return (v_nw * (s * e)) + (v_ne * (s * w)) + (v_sw * (n * e)) + (v_se * (n * w))


def warp_backward_np(x: np.ndarray, flow: np.ndarray, gout: np.ndarray, pad: str = "border",
                     need_x: bool = True, need_flow: bool = True):
    x = x.astype(f32)
    g = gout.astype(f32)
    B, C, H, W = x.shape
    t = _taps(flow, H, W, pad)
    corners = _corners(t, H, W)
    s, n, w, e = (t[k][:, None] for k in "snwe")
    gx = None
    if need_x:
        gx = np.zeros_like(x)
        bi = np.arange(B)[:, None, None, None]
        ci = np.arange(C)[None, :, None, None]
        for (cx, cy, m), wt in zip(corners, (s * e, s * w, n * e, n * w)):
            val = np.where(m[:, None], g * wt, f32(0))
            np.add.at(gx, (bi, ci, cy[:, None], cx[:, None]), val)
    gflow = None
    if need_flow:
        v_nw, v_ne, v_sw, v_se = (_gather(x, *c) for c in corners)
        tx = ((v_ne - v_nw) * s + (v_se - v_sw) * n) * g
        ty = ((v_sw - v_nw) * e + (v_se - v_ne) * w) * g
        dix = np.zeros((B, H, W), f32)
        diy = np.zeros((B, H, W), f32)
        for c in range(C):  # sequential channel accumulation, as the CPU kernel
            dix = dix + tx[:, c]
            diy = diy + ty[:, c]
        ggx = dix * t["mx"]
        ggy = diy * t["my"]
        gflow = np.stack([(ggx / f32(W - 1)) * f32(2.0), (ggy / f32(H - 1)) * f32(2.0)], 1)
    return gx, gflow


def occu_mask_bidirection_np(flow12: np.ndarray, flow21: np.ndarray, scale: float = 0.01, bias: float = 0.5,
                             warped: np.ndarray | None = None) -> np.ndarray:
    """get_occu_mask_bidirection (utils/warp_utils.py:109-117) in float32 numpy:
    ``w = flow_warp(flow21, flow12, pad="zeros")`` (or ``warped``, e.g. the
    reference's own warp output from a golden capture), ``d = flow12 + w``,
    occluded where ``|d|^2 > scale * (|flow12|^2 + |w|^2) + bias``; each
    channel sum over the 2 components is ``a + b`` as torch's ``sum(1)``, the
    Python scalars act as float32 (torch's wrapped-number promotion)."""
    f = flow12.astype(f32)
    w = warp_forward_np(flow21, flow12, "zeros") if warped is None else warped.astype(f32)
    d = f + w
    mag = (f[:, 0] * f[:, 0] + f[:, 1] * f[:, 1]) + (w[:, 0] * w[:, 0] + w[:, 1] * w[:, 1])
    th = f32(scale) * mag + f32(bias)
    return ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) > th)[:, None].astype(f32)


def occu_bidirection_margin(flow12: np.ndarray, flow21: np.ndarray, scale: float = 0.01,
                            bias: float = 0.5) -> np.ndarray:
    """|  |d|^2 - threshold  | per pixel (float64): where the mask decision is
    within rounding of the threshold, two correct implementations may differ."""
    f = flow12.astype(np.float64)
    w = warp_forward_np(flow21, flow12, "zeros").astype(np.float64)
    d = f + w
    th = scale * ((f ** 2).sum(1) + (w ** 2).sum(1)) + bias
    return np.abs((d ** 2).sum(1) - th)[:, None]


def warp_bytes(B: int, C: int, H: int, W: int, backward: bool = False, need_x: bool = True) -> int:
    """Algorithmic HBM bytes."""
    if not backward:
        per_px = 2 * C + 2
    else:
        per_px = (3 * C + 4) if need_x else (2 * C + 4)
    return 4 * B * H * W * per_px
