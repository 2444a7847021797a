"""Decoder flow upsampling.

* ``upsample_flow``: the reference's ``F.interpolate(flow * k, scale_factor=k,
  mode="bilinear", align_corners=True)`` (models/pwclite.py:299-301 between
  levels, k = 2; the x4 output flows without the learned upsampler) as one HIP
  op per direction (csrc/upsample.hip): the scale is folded into the taps and
  the backward is a deterministic gather instead of ATen's atomic scatter.
* ``upsample_warp``: that x2 upsampling fused with the decoder's warp of x2 at
  the upsampled flow (pwclite.py:299-302), one forward launch for both.
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


class ConvexUpsamplePyramidFunction(Function):
    """Every decoder level's convex x4 upsampling in one launch each way."""

    @staticmethod
    def forward(ctx, factor, mask_scale, n, *tensors):
        flows, masks = list(tensors[:n]), list(tensors[n:])
        ctx.factor, ctx.mask_scale, ctx.n = factor, mask_scale, n
        ctx.save_for_backward(*flows, *masks)
        return tuple(ops.convex_upsample_pyramid(flows, masks, factor, mask_scale))

    @staticmethod
    def backward(ctx, *grad_outs):
        n = ctx.n
        saved = ctx.saved_tensors
        flows, masks = list(saved[:n]), list(saved[n:])
        need_f = any(ctx.needs_input_grad[3:3 + n])
        need_m = any(ctx.needs_input_grad[3 + n:3 + 2 * n])
        go = [g if g is not None else torch.zeros((f.shape[0], 2, ctx.factor * f.shape[2], ctx.factor * f.shape[3]),
                                                  device=f.device) for g, f in zip(grad_outs, flows)]
        gfs, gms = ops.convex_upsample_pyramid_backward(flows, masks, go, ctx.factor, ctx.mask_scale, need_f, need_m)
        return (None, None, None, *(gfs if gfs is not None else [None] * n),
                *(gms if gms is not None else [None] * n))


def convex_upsample_pyramid(flows, masks, factor: int = 4, mask_scale: float = 0.25):
    """``[convex_upsample(f, m, factor, mask_scale) for f, m in zip(flows, masks)]``
    in one launch forward and one (+ one gather) backward."""
    return list(ConvexUpsamplePyramidFunction.apply(int(factor), float(mask_scale), len(flows), *flows, *masks))


class UpsampleWarpFunction(Function):
    """The decoder's ``flow = upsample_flow(coarse, 2); x2_warp = flow_warp(x2, flow)``
    (pwclite.py:299-302) with ONE forward launch (``ops.warp_forward_up``: the
    same numbers). Backward: the warp backward at the upsampled flow, its flow
    gradient added to the one the upsampled flow receives from its other uses,
    then the upsampling backward -- what autograd does for the two-op form."""

    @staticmethod
    def forward(ctx, coarse, x, pad):
        up, out = ops.warp_forward_up(x, coarse, pad)
        ctx.pad = pad
        ctx.save_for_backward(x, up)
        return up, out

    @staticmethod
    def backward(ctx, g_up, g_out):
        x, up = ctx.saved_tensors
        need_c, need_x = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gx = gflow = None
        if g_out is not None and (need_x or need_c):
            gx, gflow = ops.warp_backward(x, up, g_out, ctx.pad, need_x=need_x, need_flow=need_c)
        gc = None
        if need_c:
            if g_up is not None and gflow is not None:  # the add inside the upsampling backward
                gc = ops.flow_upsample_backward(g_up, 2, gflow)
            elif g_up is not None or gflow is not None:
                gc = ops.flow_upsample_backward(g_up if g_up is not None else gflow, 2)
        return gc, gx, None


def upsample_warp(coarse: torch.Tensor, x: torch.Tensor, pad: str = "border"):
    """``(up, flow_warp(x, up))`` with ``up = F.interpolate(coarse * 2, scale_factor=2,
    mode="bilinear", align_corners=True)`` (pwclite.py:299-302), one launch forward."""
    return UpsampleWarpFunction.apply(coarse, x, pad)


def upsample_flow(flow: torch.Tensor, factor: int) -> torch.Tensor:
    """``F.interpolate(flow * factor, scale_factor=factor, mode="bilinear", align_corners=True)``."""
    return FlowUpsampleFunction.apply(flow, int(factor))
