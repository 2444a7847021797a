"""Fused correlation epilogue: the decoder's

    cost = leakyRELU(corr(x1, x2_warp))                    (pwclite.py:307-308)
    x = cat([cost, (mask cost,) conv_1x1(x1), flow], 1)    (pwclite.py:364-366)

as one autograd op. The correlation kernel writes LeakyReLU(corr) straight
into its channel slice of the concat buffer (usf_corr_fwd_ex_f32: output batch
stride + activation epilogue), so the 81-channel cost map is neither written
twice (activation pass) nor copied (cat). Backward reads its gradient from the
concat gradient's slice (batch stride) and applies the LeakyReLU derivative:
from the sign mask the forward wrote (the tiled kernel's epilogue; at the
small levels the small-image kernel's, or the channel split's reduce where a
row is too wide for it), inside the backward
kernel's gradient loads (usf_corr_bwd_ex_f32) at every level; the extras'
gradients are views.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from . import ops


class CorrLeakyCatFunction(Function):
    @staticmethod
    def forward(ctx, max_displacement, slope, n_pairs, *tensors):
        pairs = [(tensors[2 * i], tensors[2 * i + 1]) for i in range(n_pairs)]
        extras = tensors[2 * n_pairs:]
        B, _, H, W = pairs[0][0].shape
        K2 = (2 * max_displacement + 1) ** 2
        ctot = K2 * n_pairs + sum(e.shape[1] for e in extras)
        buf = torch.empty((B, ctot, H, W), device=pairs[0][0].device, dtype=torch.float32)
        off = 0
        masks = []
        for a, b in pairs:
            m = ops.corr_act_mask(B, H, W, max_displacement, a.device, C=a.shape[1])
            ops.corr_forward_ex(a, b, max_displacement, buf[:, off:off + K2], slope, act_mask=m)
            masks.append(m)
            off += K2
        for e in extras:
            buf[:, off:off + e.shape[1]].copy_(e)
            off += e.shape[1]
        ctx.md, ctx.slope, ctx.n_pairs, ctx.k2 = max_displacement, slope, n_pairs, K2
        ctx.extra_ch = [e.shape[1] for e in extras]
        # per pair: with add_mask_corr the pairs can differ in C, so one pair's
        # forward may split its channel loop (no mask) while the other's writes one
        ctx.mask_idx = [i for i, m in enumerate(masks) if m is not None]
        ctx.save_for_backward(*[t for p in pairs for t in p], *[masks[i] for i in ctx.mask_idx], buf)
        return buf

    @staticmethod
    def backward(ctx, gbuf):
        saved = ctx.saved_tensors
        buf = saved[-1]
        masks = [None] * ctx.n_pairs
        for j, i in enumerate(ctx.mask_idx):
            masks[i] = saved[2 * ctx.n_pairs + j]
        grads = []
        off = 0
        gbuf = gbuf if gbuf.is_contiguous() else gbuf.contiguous()
        for i in range(ctx.n_pairs):
            a, b = saved[2 * i], saved[2 * i + 1]
            need_a = ctx.needs_input_grad[3 + 2 * i]
            need_b = ctx.needs_input_grad[4 + 2 * i]
            ga, gb = ops.corr_backward_ex(a, b, gbuf[:, off:off + ctx.k2], ctx.md, need_a, need_b,
                                          act_out=buf[:, off:off + ctx.k2], leaky_slope=ctx.slope,
                                          act_mask=masks[i])
            grads += [ga, gb]
            off += ctx.k2
        for c in ctx.extra_ch:
            grads.append(gbuf[:, off:off + c])
            off += c
        return (None, None, None, *grads)


def corr_leaky_cat(pairs, extras, max_displacement: int = 4, slope: float = 0.1) -> torch.Tensor:
    """cat([leaky(corr(a, b)) for a, b in pairs] + extras, dim=1), fused."""
    flat = [t for p in pairs for t in p]
    return CorrLeakyCatFunction.apply(int(max_displacement), float(slope), len(pairs), *flat, *extras)
