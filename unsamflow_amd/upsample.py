"""Decoder flow upsampling.

* ``upsample_flow``: the reference's ``F.interpolate(flow * k, scale_factor=k,
  mode="bilinear", align_corners=True)`` (models/pwclite.py:299-301 between
  levels, k = 2; the x4 output flows without the learned upsampler) as one HIP
  op per direction (csrc/upsample.hip): the scale is folded into the taps and
  the backward is a deterministic gather instead of ATen's atomic scatter.
* ``convex_upsample``: the learned RAFT-style upsampler of the output flows,
  ``UpFlowNetwork.upsample_flow(flow, 0.25 * convs(feat))`` (pwclite.py:
  140-166; on in kitti_base / sintel_base), as one HIP pass forward and a
  pass + 9-tap gather backward (csrc/convex.hip) instead of torch's softmax /
  unfold / broadcast-multiply / sum / permute chain.
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


class ConvexUpsampleFunction(Function):
    @staticmethod
    def forward(ctx, flow, mask, factor, mask_scale):
        ctx.factor, ctx.mask_scale = factor, mask_scale
        ctx.save_for_backward(flow, mask)
        return ops.convex_upsample(flow, mask, factor, mask_scale)

    @staticmethod
    def backward(ctx, grad_out):
        flow, mask = ctx.saved_tensors
        gf, gm = ops.convex_upsample_backward(flow, mask, grad_out, ctx.factor, ctx.mask_scale,
                                              ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return gf, gm, None, None


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor, factor: int = 4, mask_scale: float = 0.25) -> torch.Tensor:
    """``UpFlowNetwork.upsample_flow(flow, mask_scale * mask)``: flow [B,2,H,W], mask
    [B,9*f*f,H,W] (the convs' raw output) -> [B,2,f*H,f*W] (pwclite.py:148-166)."""
    return ConvexUpsampleFunction.apply(flow, mask, int(factor), float(mask_scale))


def upsample_flow(flow: torch.Tensor, factor: int) -> torch.Tensor:
    """``F.interpolate(flow * factor, scale_factor=factor, mode="bilinear", align_corners=True)``."""
    return FlowUpsampleFunction.apply(flow, int(factor))
