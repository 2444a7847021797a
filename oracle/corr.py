"""TEST INFRASTRUCTURE ONLY — correlation oracle (see oracle/__init__.py).

Restates the reference's local correlation:

* forward — ``models/correlation_native.py:13-23``: zero-pad x2 by d on all
  four sides (:16), for i (vertical) and j (horizontal) in 0..2d take the
  shifted window x2p[:, :, i:i+H, j:j+W] (:18-20), channel-mean of its product
  with x1 (:21), concatenated in (i, j) row-major order (:23).
* backward — the gradients autograd derives for that graph, identical to the
  CUDA plugin's correlation_backward_input1/2 (correlation_cuda_kernel.cu:
  116-207, 209-300; division by nelems = C at :200, :293):
    gx1[c,y,x] = (1/C) sum_k g[k,y,x] * X2[c, y+dy_k, x+dx_k]
    gx2[c,y,x] = (1/C) sum_k G[k, y-dy_k, x-dx_k] * X1[c, y-dy_k, x-dx_k]

Two flavours: numpy (float64 accumulation available, used for the parity
truth and gradcheck-style tests) and torch-CPU (the timed CPU baseline and the
CPU harness).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _shifts(d: int):
    K = 2 * d + 1
    for i in range(K):
        for j in range(K):
            yield i * K + j, i, j


def corr_forward_np(x1: np.ndarray, x2: np.ndarray, d: int = 4, acc_dtype=np.float64) -> np.ndarray:
    """[B,C,H,W] x 2 -> [B,(2d+1)^2,H,W] (correlation_native.py:13-23)."""
    B, C, H, W = x1.shape
    K = 2 * d + 1
    a = x1.astype(acc_dtype)
    x2p = np.pad(x2.astype(acc_dtype), ((0, 0), (0, 0), (d, d), (d, d)))
    out = np.empty((B, K * K, H, W), dtype=acc_dtype)
    for k, i, j in _shifts(d):
        out[:, k] = (a * x2p[:, :, i:i + H, j:j + W]).mean(axis=1)
    return out


def corr_backward_np(x1: np.ndarray, x2: np.ndarray, g: np.ndarray, d: int = 4, acc_dtype=np.float64):
    """(gx1, gx2) for grad_output g [B,(2d+1)^2,H,W]."""
    B, C, H, W = x1.shape
    a = x1.astype(acc_dtype)
    x2p = np.pad(x2.astype(acc_dtype), ((0, 0), (0, 0), (d, d), (d, d)))
    gg = g.astype(acc_dtype)
    gx1 = np.zeros((B, C, H, W), dtype=acc_dtype)
    gx2p = np.zeros_like(x2p)
    for k, i, j in _shifts(d):
        gk = gg[:, k:k + 1] / C
        gx1 += gk * x2p[:, :, i:i + H, j:j + W]
        gx2p[:, :, i:i + H, j:j + W] += gk * a
    return gx1, gx2p[:, :, d:d + H, d:d + W]


def corr_backward_torch64(x1: torch.Tensor, x2: torch.Tensor, g: torch.Tensor, d: int = 4):
    """corr_backward_np in torch-CPU float64 (same formulas, multi-threaded): the
    checker for full-size shapes, e.g. the decoder's L4 site at batch 16."""
    B, C, H, W = x1.shape
    a = x1.double()
    x2p = F.pad(x2.double(), [d] * 4)
    gg = g.double() / C
    gx1 = torch.zeros((B, C, H, W), dtype=torch.float64)
    gx2p = torch.zeros_like(x2p)
    for k, i, j in _shifts(d):
        gk = gg[:, k:k + 1]
        gx1 += gk * x2p[:, :, i:i + H, j:j + W]
        gx2p[:, :, i:i + H, j:j + W] += gk * a
    return gx1, gx2p[:, :, d:d + H, d:d + W]


def corr_forward_torch64(x1: torch.Tensor, x2: torch.Tensor, d: int = 4) -> torch.Tensor:
    """corr_forward_np in torch-CPU float64 (correlation_native.py:13-23, multi-threaded):
    the checker for full-size forwards, e.g. the decoder's L4 site at batch 16."""
    B, C, H, W = x1.shape
    K = 2 * d + 1
    a = x1.double()
    x2p = F.pad(x2.double(), [d] * 4)
    out = torch.empty((B, K * K, H, W), dtype=torch.float64)
    for k, i, j in _shifts(d):
        out[:, k] = (a * x2p[:, :, i:i + H, j:j + W]).mean(dim=1)
    return out


def corr_forward_torch(x1: torch.Tensor, x2: torch.Tensor, d: int = 4) -> torch.Tensor:
    """torch-CPU restatement of correlation_native.py:13-23 (differentiable by autograd)."""
    B, C, H, W = x1.shape
    K = 2 * d + 1
    x2p = F.pad(x2, [d] * 4)
    return torch.cat(
        [torch.mean(x1 * x2p[:, :, i:i + H, j:j + W], 1, keepdim=True) for i in range(K) for j in range(K)],
        1,
    )


class OracleCorrelation(torch.nn.Module):
    """CPU module with the native Correlation's behaviour (no parameters)."""

    def __init__(self, max_displacement=4, *args, **kwargs):
        super().__init__()
        self.max_displacement = max_displacement

    def forward(self, x1, x2):
        return corr_forward_torch(x1, x2, self.max_displacement)


def corr_bytes(B: int, C: int, H: int, W: int, K2: int = 81, backward: bool = False) -> int:
    """Algorithmic HBM bytes: inputs read once, outputs written once."""
    per_px = (K2 + 4 * C) if backward else (2 * C + K2)
    return 4 * B * H * W * per_px


def corr_flops(B: int, C: int, H: int, W: int, K2: int = 81, backward: bool = False) -> int:
    return (4 if backward else 2) * K2 * C * B * H * W
