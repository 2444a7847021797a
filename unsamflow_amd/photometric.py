"""Fused photometric loss: the per-scale, per-direction
``loss_photomatric(im1_s, flow_warp(im2_s, flow), vis_mask)`` of
losses/flow_loss.py:127-148 (L1 + SSIM, loss_blocks.py:53-72) as one autograd
op (unsamflow_amd/csrc/photo.hip): no warped image, SSIM maps or intermediate
gradients in HBM, and the gradient reaches only the flow (the images and the
thresholded occlusion mask carry none, as in the reference). When the flow needs
a gradient, the forward pass also writes the per-pixel gradient basis (the loss
is linear in its L1 and SSIM sums), so the backward is one dense pass.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from . import ops


class PhotometricLossFunction(Function):
    @staticmethod
    def forward(ctx, flow, src, tgt, mask, pad, w_l1, w_ssim):
        need = ctx.needs_input_grad[0]
        out, basis = ops.photo_loss_forward(src, tgt, mask, flow, pad, w_l1, w_ssim, need_grad=need)
        if need:
            ctx.save_for_backward(basis, out)
        return out[0].clone()

    @staticmethod
    def backward(ctx, grad_loss):
        gflow = None
        if ctx.needs_input_grad[0]:
            basis, out = ctx.saved_tensors
            gflow = ops.photo_loss_backward(basis, out, grad_loss)
        return gflow, None, None, None, None, None, None


def photometric_loss(flow: torch.Tensor, src: torch.Tensor, tgt: torch.Tensor, mask: torch.Tensor,
                     pad: str = "border", w_l1: float = 0.15, w_ssim: float = 0.85) -> torch.Tensor:
    """``loss_photomatric(tgt, flow_warp(src, flow, pad), mask)`` with w_ternary = 0."""
    if src.requires_grad or tgt.requires_grad:
        raise NotImplementedError("the fused photometric loss differentiates w.r.t. the flow only")
    return PhotometricLossFunction.apply(flow, src, tgt, mask.detach(), pad, float(w_l1), float(w_ssim))


class PhotometricPairFunction(Function):
    """Both directions of a with_bk scale in one launch: returns [2] losses
    (direction 0: im1 vs warp(im2, flow[:, :2]) under mask1; direction 1: im2
    vs warp(im1, flow[:, 2:]) under mask2); the gradient is [B,4,H,W]."""

    @staticmethod
    def forward(ctx, flow, im1, im2, mask1, mask2, pad, w_l1, w_ssim):
        need = ctx.needs_input_grad[0]
        out, basis = ops.photo_loss_pair_forward(flow, im1, im2, mask1, mask2, pad, w_l1, w_ssim,
                                                 need_grad=need)
        if need:
            ctx.save_for_backward(basis, out)
        return out.view(2, 3)[:, 0].clone()

    @staticmethod
    def backward(ctx, grad_losses):
        gflow = None
        if ctx.needs_input_grad[0]:
            basis, out = ctx.saved_tensors
            gflow = ops.photo_loss_backward(basis, out, grad_losses)
        return gflow, None, None, None, None, None, None, None


def photometric_loss_pair(flow: torch.Tensor, im1: torch.Tensor, im2: torch.Tensor, mask1: torch.Tensor,
                          mask2: torch.Tensor, pad: str = "border", w_l1: float = 0.15,
                          w_ssim: float = 0.85) -> torch.Tensor:
    """``[loss_photomatric(im1, flow_warp(im2, flow[:, :2]), mask1),
    loss_photomatric(im2, flow_warp(im1, flow[:, 2:]), mask2)]`` (flow_loss.py:130-131)
    in one launch; ``flow`` is the [B,4,H,W] forward+backward flow."""
    if im1.requires_grad or im2.requires_grad:
        raise NotImplementedError("the fused photometric loss differentiates w.r.t. the flow only")
    return PhotometricPairFunction.apply(flow, im1, im2, mask1.detach(), mask2.detach(), pad, float(w_l1),
                                         float(w_ssim))


class PhotometricPyramidFunction(Function):
    """The with_bk pairs of up to 4 loss scales in one launch (the largest
    first): returns [nscale, 2] losses; the gradient w.r.t. each scale's
    [B,4,H,W] flow comes from one backward launch for all scales."""

    @staticmethod
    def forward(ctx, pad, w_l1, w_ssim, n, *tensors):
        flows, im1s, im2s, m1s, m2s = (list(tensors[i * n:(i + 1) * n]) for i in range(5))
        need = any(ctx.needs_input_grad[4:4 + n])
        out, bases = ops.photo_loss_pyramid_forward(flows, im1s, im2s, m1s, m2s, pad, w_l1, w_ssim, need_grad=need)
        ctx.n = n
        if need:
            ctx.save_for_backward(out, *bases)
        return out[:, 0::3].clone()

    @staticmethod
    def backward(ctx, grad_losses):
        n = ctx.n
        grads = [None] * (4 + 5 * n)
        if any(ctx.needs_input_grad[4:4 + n]):
            out, *bases = ctx.saved_tensors
            gflows = ops.photo_loss_pyramid_backward(bases, out, grad_losses)
            for k in range(n):
                if ctx.needs_input_grad[4 + k]:
                    grads[4 + k] = gflows[k]
        return tuple(grads)


def photometric_loss_pyramid(flows, im1s, im2s, masks1, masks2, pad: str = "border", w_l1: float = 0.15,
                             w_ssim: float = 0.85) -> torch.Tensor:
    """``[photometric_loss_pair(flows[k], im1s[k], im2s[k], masks1[k], masks2[k]) for k]``
    (flow_loss.py:120-148's scale loop, with_bk) as [nscale, 2] from ONE forward
    launch and one backward launch; the same numbers as the per-scale calls."""
    if any(t.requires_grad for t in list(im1s) + list(im2s)):
        raise NotImplementedError("the fused photometric loss differentiates w.r.t. the flow only")
    n = len(flows)
    return PhotometricPyramidFunction.apply(pad, float(w_l1), float(w_ssim), n, *flows, *im1s, *im2s,
                                            *[m.detach() for m in masks1], *[m.detach() for m in masks2])
