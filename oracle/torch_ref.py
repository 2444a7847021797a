"""TEST INFRASTRUCTURE ONLY — torch-CPU hot-path ops with reference semantics
(see oracle/__init__.py). Injected into the PWCLite/loss harness for the CPU
tests (incl. the gloo DDP tests) and for bench.py's CPU baseline; never used by
the product path.

* ``OracleCorrelation`` — correlation_native.py:13-23 (oracle/corr.py).
* ``oracle_flow_warp`` — utils/warp_utils.py:97-106: pixel grid + flow,
  norm_grid (:16-23), torch ``grid_sample(bilinear, align_corners=True)``.
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
