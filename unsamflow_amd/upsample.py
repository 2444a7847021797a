"""Decoder flow upsampling: the reference's
``F.interpolate(flow * k, scale_factor=k, mode="bilinear", align_corners=True)``
(models/pwclite.py:299-301 between levels, k = 2; the x4 output flows) as one
HIP op per direction (csrc/upsample.hip): the scale is folded into the taps
and the backward is a deterministic gather instead of ATen's atomic scatter.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from . import ops


class FlowUpsampleFunction(Function):
    @staticmethod
    def forward(ctx, flow, factor):
        ctx.factor = factor
        return ops.flow_upsample(flow, factor)

    @staticmethod
    def backward(ctx, grad_out):
        return ops.flow_upsample_backward(grad_out, ctx.factor), None


def upsample_flow(flow: torch.Tensor, factor: int) -> torch.Tensor:
    """``F.interpolate(flow * factor, scale_factor=factor, mode="bilinear", align_corners=True)``."""
    return FlowUpsampleFunction.apply(flow, int(factor))
