"""TEST INFRASTRUCTURE ONLY — CPU restatement of the learned (convex) flow
upsampler, the parity oracle for ``usf_convex_upsample_*`` (csrc/convex.hip).

Reference: ``UpFlowNetwork`` in models/pwclite.py:140-166 (RAFT-style):
``forward`` scales the convs' output by 0.25 (:163-165); ``upsample_flow``
(:148-160) views the mask as [N,1,9,f,f,H,W], softmaxes over the 9
neighbours (:152-153), unfolds ``f * flow`` over a zero-padded 3x3
neighbourhood (:155-156), takes the weighted sum over the neighbours
(:158) and interleaves the f x f sub-pixels into [N,2,fH,fW] (:159-160).

Computed in float64 numpy (the kernels are fp32; tests compare with a
tolerance). Pinned by ``tests/golden/convex_*.npz``, captured from the
reference's own ``upsample_flow`` + autograd (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np


def _weights(mask: np.ndarray, f: int, mask_scale: float) -> np.ndarray:
    """softmax(mask_scale * mask viewed [N,9,f,f,H,W], over the 9) (pwclite.py:152-153)."""
    N, _, H, W = mask.shape
    m = mask_scale * mask.astype(np.float64).reshape(N, 9, f, f, H, W)
    m = m - m.max(axis=1, keepdims=True)
    e = np.exp(m)
    return e / e.sum(axis=1, keepdims=True)


def _patches(flow: np.ndarray, f: int) -> np.ndarray:
    """unfold(f * flow, [3, 3], padding=1) viewed [N,2,9,H,W] (pwclite.py:155-156)."""
    N, C, H, W = flow.shape
    fp = np.pad(f * flow.astype(np.float64), ((0, 0), (0, 0), (1, 1), (1, 1)))
    return np.stack([fp[:, :, ky:ky + H, kx:kx + W] for ky in range(3) for kx in range(3)], axis=2)


def convex_upsample_np(flow: np.ndarray, mask: np.ndarray, factor: int = 4,
                       mask_scale: float = 0.25) -> np.ndarray:
    """UpFlowNetwork.upsample_flow(flow, mask_scale * mask) -> [N,2,fH,fW] (pwclite.py:148-166)."""
    f = int(factor)
    N, C, H, W = flow.shape
    w = _weights(mask, f, mask_scale)                            # N,9,f,f,H,W
    v = _patches(flow, f)                                        # N,2,9,H,W
    up = np.einsum("nkijyx,nckyx->ncijyx", w, v)                 # :158
    return up.transpose(0, 1, 4, 2, 5, 3).reshape(N, C, f * H, f * W)  # :159-160


def convex_upsample_backward_np(flow: np.ndarray, mask: np.ndarray, grad_out: np.ndarray,
                                factor: int = 4, mask_scale: float = 0.25):
    """(grad_flow [N,2,H,W], grad_mask [N,9ff,H,W] w.r.t. the raw mask)."""
    f = int(factor)
    N, C, H, W = flow.shape
    w = _weights(mask, f, mask_scale)
    v = _patches(flow, f)
    G = grad_out.astype(np.float64).reshape(N, C, H, f, W, f).transpose(0, 1, 3, 5, 2, 4)  # N,2,f,f,H,W
    dp = np.einsum("ncijyx,nckyx->nkijyx", G, v)                 # d loss / d weights
    dot = (w * dp).sum(axis=1, keepdims=True)
    grad_mask = (mask_scale * w * (dp - dot)).reshape(N, 9 * f * f, H, W)   # softmax backward
    gv = np.einsum("nkijyx,ncijyx->nckyx", w, G)                 # d loss / d patches
    gp = np.zeros((N, C, H + 2, W + 2))
    for ky in range(3):
        for kx in range(3):
            gp[:, :, ky:ky + H, kx:kx + W] += gv[:, :, ky * 3 + kx]       # unfold's backward (col2im)
    return f * gp[:, :, 1:-1, 1:-1], grad_mask


def convex_bytes(B: int, H: int, W: int, factor: int = 4, backward: bool = False) -> int:
    """Algorithmic HBM bytes: inputs read once, outputs written once (fp32).
    Forward: flow (2) + mask (9 f^2) read, out (2 f^2) written, per low-res pixel.
    Backward: flow, mask, grad_out read; grad_flow, grad_mask written."""
    ff = factor * factor
    per = 2 + 9 * ff + 2 * ff if not backward else 2 + 9 * ff + 2 * ff + 2 + 9 * ff
    return 4 * B * H * W * per
