"""Fused photometric loss: the per-scale, per-direction
``loss_photomatric(im1_s, flow_warp(im2_s, flow), vis_mask)`` of
losses/flow_loss.py:127-148 (L1 + SSIM, loss_blocks.py:53-72) as one autograd
op over two HIP kernels (unsamflow_amd/csrc/photo.hip): no warped image, SSIM
maps or intermediate gradients in HBM, and the gradient reaches only the flow
(the images and the thresholded occlusion mask carry none, as in the reference).
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from . import ops


class PhotometricLossFunction(Function):
    @staticmethod
    def forward(ctx, flow, src, tgt, mask, pad, w_l1, w_ssim):
        out = ops.photo_loss_forward(src, tgt, mask, flow, pad, w_l1, w_ssim)
        ctx.save_for_backward(flow, src, tgt, mask, out)
        ctx.pad = pad
        return out[0].clone()

    @staticmethod
    def backward(ctx, grad_loss):
        flow, src, tgt, mask, out = ctx.saved_tensors
        gflow = None
        if ctx.needs_input_grad[0]:
            gflow = ops.photo_loss_backward(src, tgt, mask, flow, out, grad_loss, ctx.pad)
        return gflow, None, None, None, None, None, None


def photometric_loss(flow: torch.Tensor, src: torch.Tensor, tgt: torch.Tensor, mask: torch.Tensor,
                     pad: str = "border", w_l1: float = 0.15, w_ssim: float = 0.85) -> torch.Tensor:
    """``loss_photomatric(tgt, flow_warp(src, flow, pad), mask)`` with w_ternary = 0."""
    if src.requires_grad or tgt.requires_grad:
        raise NotImplementedError("the fused photometric loss differentiates w.r.t. the flow only")
    return PhotometricLossFunction.apply(flow, src, tgt, mask.detach(), pad, float(w_l1), float(w_ssim))
