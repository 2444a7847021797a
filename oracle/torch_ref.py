"""TEST INFRASTRUCTURE ONLY — torch-CPU hot-path ops with reference semantics
(see oracle/__init__.py). Injected into the PWCLite/loss harness for the CPU
tests (incl. the gloo DDP tests) and for bench.py's CPU baseline; never used by
the product path.

* ``OracleCorrelation`` — correlation_native.py:13-23 (oracle/corr.py).
* ``oracle_flow_warp`` — utils/warp_utils.py:97-106: pixel grid + flow,
  norm_grid (:16-23), torch ``grid_sample(bilinear, align_corners=True)``.
* ``oracle_corresponding_map`` / ``oracle_occu_mask_backward`` —
  warp_utils.py:26-94 / :120-126: bilinear forward splat with ``scatter_add_``
  (corner order and validity tests as the reference), threshold < th.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .corr import OracleCorrelation  # noqa: F401


def oracle_flow_warp(x: torch.Tensor, flow12: torch.Tensor, pad: str = "border", mode: str = "bilinear"):
    B, _, H, W = x.size()
    xs = torch.arange(W, device=x.device, dtype=x.dtype).view(1, 1, W).expand(B, H, W)
    ys = torch.arange(H, device=x.device, dtype=x.dtype).view(1, H, 1).expand(B, H, W)
    vx = xs + flow12[:, 0]
    vy = ys + flow12[:, 1]
    grid = torch.stack([2.0 * vx / (W - 1) - 1.0, 2.0 * vy / (H - 1) - 1.0], dim=-1)
    return F.grid_sample(x, grid, mode=mode, padding_mode=pad, align_corners=True)


def oracle_occu_mask_bidirection(flow12, flow21, scale=0.01, bias=0.5):
    w = oracle_flow_warp(flow21, flow12, pad="zeros")
    diff = flow12 + w
    mag = (flow12 * flow12).sum(1, keepdim=True) + (w * w).sum(1, keepdim=True)
    return ((diff * diff).sum(1, keepdim=True) > scale * mag + bias).float()


def oracle_corresponding_map(data: torch.Tensor) -> torch.Tensor:
    """get_corresponding_map (warp_utils.py:26-94): data = target coords [B,2,H,W]."""
    B, _, H, W = data.size()
    x = data[:, 0].reshape(B, -1)
    y = data[:, 1].reshape(B, -1)
    x0 = torch.floor(x)
    y0 = torch.floor(y)
    x1 = x0 + 1
    y1 = y0 + 1
    xw, yn = x0.clamp(0, W - 1), y0.clamp(0, H - 1)
    xe, ys = x1.clamp(0, W - 1), y1.clamp(0, H - 1)
    out = torch.zeros(B, H * W, dtype=data.dtype, device=data.device)
    idx, val = [], []
    for cx, cy, okx, oky in ((xe, ys, x1 == xe, y1 == ys), (xe, yn, x1 == xe, y0 == yn),
                             (xw, ys, x0 == xw, y1 == ys), (xw, yn, x0 == xw, y0 == yn)):
        wgt = (1 - torch.abs(x - cx)) * (1 - torch.abs(y - cy))
        idx.append(cx + cy * W)
        val.append(torch.where(okx & oky, wgt, torch.zeros_like(wgt)))
    out.scatter_add_(1, torch.cat(idx, 1).long(), torch.cat(val, 1))
    return out.view(B, 1, H, W)


def oracle_occu_mask_backward(flow21: torch.Tensor, th: float = 0.2) -> torch.Tensor:
    """get_occu_mask_backward (warp_utils.py:120-126)."""
    B, _, H, W = flow21.size()
    xs = torch.arange(W, device=flow21.device, dtype=flow21.dtype).view(1, 1, W).expand(B, H, W)
    ys = torch.arange(H, device=flow21.device, dtype=flow21.dtype).view(1, H, 1).expand(B, H, W)
    base = torch.stack([xs, ys], 1)
    corr_map = oracle_corresponding_map(base + flow21)
    return (corr_map.clamp(min=0.0, max=1.0) < th).float()
