"""Unsupervised flow loss — the second caller of the hot path
(losses/flow_loss.py + losses/loss_blocks.py), rebuilt for the benchmark.

``unFlowLoss(cfg)(pyramid_flows, img1, img2)`` follows
``unFlowLoss.loss_one_pair`` (flow_loss.py:83-259): occlusion masks from the
finest backward flow (``get_occu_mask_backward`` when ``occ_from_back``, else
the bidirectional check), nearest-resized per scale; per scale with
``w_ph_scales[i] > 0``: area-downsample both images, **flow_warp** them by the
two flow halves (``flow[:, :2]`` / ``flow[:, 2:]``, :130-131), occlusion-aware
photometric loss (L1 + SSIM + ternary, :33-50) averaged over the two
directions; edge-aware 1st/2nd-order smoothness at scale 0 when ``w_sm > 0``.
On a ROCm device with the library's warp and ``w_ternary == 0`` the warp +
L1 + SSIM of each scale and direction is one fused autograd op
(unsamflow_amd.photometric); ``fused_photometric=False``
or an injected ``warp_fn`` keeps the torch composition.
Returns ``(loss[None], l_ph[None], l_sm[None], flow_mean[None], vis1, vis2)``.

``smooth_type == "homography"`` needs OpenCV RANSAC on the host
(loss_blocks.py:125-200) and is not supported (not on the hot path; the base
configs use ``w_sm = 0``).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.nn as nn
import torch.nn.functional as F


def _avg3(t):
    return F.avg_pool2d(t, 3, 1, 0)


def SSIM(x, y, md=1):
    """Per-pixel (1 - SSIM)/2 over 3x3 valid windows (loss_blocks.py:53-72)."""
    if md != 1:
        x_pool = lambda t: F.avg_pool2d(t, 2 * md + 1, 1, 0)  # noqa: E731
    else:
        x_pool = _avg3
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    mu_x, mu_y = x_pool(x), x_pool(y)
    mu_xy = mu_x * mu_y
    mu_x2, mu_y2 = mu_x.pow(2), mu_y.pow(2)
    sig_x = x_pool(x * x) - mu_x2
    sig_y = x_pool(y * y) - mu_y2
    sig_xy = x_pool(x * y) - mu_xy
    num = (2 * mu_xy + C1) * (2 * sig_xy + C2)
    den = (mu_x2 + mu_y2 + C1) * (sig_x + sig_y + C2)
    return torch.clamp((1 - num / den) / 2, 0, 1)


def TernaryLoss(im, im_warp, max_distance=1):
    """Soft census-transform distance (loss_blocks.py:12-50)."""
    p = 2 * max_distance + 1

    def census(img):
        gray = (img[:, 0] * 0.2989 + img[:, 1] * 0.5870 + img[:, 2] * 0.1140).unsqueeze(1) * 255
        eye = torch.eye(p * p, dtype=img.dtype, device=img.device).view(p * p, 1, p, p)
        d = F.conv2d(gray, eye, padding=max_distance) - gray
        return d / torch.sqrt(0.81 + d * d)

    t1, t2 = census(im), census(im_warp)
    dist = (t1 - t2).pow(2)
    dist = (dist / (0.1 + dist)).mean(1, keepdim=True)
    n, _, h, w = im.shape
    mask = F.pad(torch.ones(n, 1, h - 2 * max_distance, w - 2 * max_distance, dtype=im.dtype, device=im.device),
                 [max_distance] * 4)
    return dist * mask


def gradient(data):
    return data[..., :, 1:] - data[..., :, :-1], data[..., 1:, :] - data[..., :-1, :]


def _edge_weights(image=None, alpha=10, full_seg=None):
    if full_seg is not None:
        return ((full_seg[..., :, 1:] - full_seg[..., :, :-1]) == 0).float(), \
            ((full_seg[..., 1:, :] - full_seg[..., :-1, :]) == 0).float()
    dx, dy = gradient(image)
    return torch.exp(-dx.abs().mean(1, keepdim=True) * alpha), torch.exp(-dy.abs().mean(1, keepdim=True) * alpha)


def smooth_grad_1st(flo, image, edge="image", **kw):
    wx, wy = _edge_weights(image, kw.get("alpha", 10), kw.get("full_seg") if edge == "full_seg" else None)
    dx, dy = gradient(flo)
    return (wx * dx.abs()).mean() / 2.0 + (wy * dy.abs()).mean() / 2.0


def smooth_grad_2nd(flo, image, edge="image", **kw):
    wx, wy = _edge_weights(image, kw.get("alpha", 10), kw.get("full_seg") if edge == "full_seg" else None)
    dx, dy = gradient(flo)
    dx2, _ = gradient(dx)
    _, dy2 = gradient(dy)
    return (wx[:, :, :, 1:] * dx2.abs()).mean() / 2.0 + (wy[:, :, 1:, :] * dy2.abs()).mean() / 2.0


def _default_warp():
    from .warp_utils import flow_warp

    return flow_warp


# every weighted loss scale's photometric pair in one launch (photometric_loss_pyramid)
PHOTO_PYRAMID = True


class unFlowLoss(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, cfg, warp_fn: Callable | None = None, occ_backward_fn: Callable | None = None,
                 occ_bidir_fn: Callable | None = None, fused_photometric: bool = True):
        super().__init__()
        self.cfg = cfg
        if "ransac_threshold" not in cfg:
            self.cfg.ransac_threshold = 3
        from . import warp_utils

        self.warp = warp_fn if warp_fn is not None else _default_warp()
        # fused photometric kernels only behind the library's own warp (an injected
        # warp -- e.g. the CPU oracle -- keeps the torch composition below)
        self.fused = warp_fn is None and fused_photometric
        self.occ_backward = occ_backward_fn or warp_utils.get_occu_mask_backward
        self.lib_occ = occ_backward_fn is None  # the library's masks: both directions in one call
        self.occ_bidir = occ_bidir_fn or (lambda f12, f21: warp_utils.get_occu_mask_bidirection(f12, f21))

    def _fused_photometric(self, flow) -> bool:
        """Fused HIP warp+L1+SSIM (unsamflow_amd.photometric) when this loss uses the
        library's own warp on a ROCm device and the photometric terms are L1/SSIM."""
        c = self.cfg
        return (self.fused and flow.is_cuda and c.w_ternary == 0 and c.w_l1 >= 0 and c.w_ssim >= 0)

    def loss_photomatric(self, im1_scaled, im1_recons, vis_mask1):
        c = self.cfg
        terms = []
        if c.w_l1 > 0:
            terms.append(c.w_l1 * (im1_scaled - im1_recons).abs() * vis_mask1)
        if c.w_ssim > 0:
            terms.append(c.w_ssim * SSIM(im1_recons * vis_mask1, im1_scaled * vis_mask1))
        if c.w_ternary > 0:
            terms.append(c.w_ternary * TernaryLoss(im1_recons * vis_mask1, im1_scaled * vis_mask1))
        return sum(t.mean() for t in terms) / (vis_mask1.mean() + 1e-6)

    def loss_smooth(self, flow, im1_scaled, **kw):
        fn = {"2nd": smooth_grad_2nd, "1st": smooth_grad_1st}[self.cfg.smooth_type]
        if "smooth_edge" not in self.cfg or self.cfg.smooth_edge == "image":
            return fn(flow, im1_scaled, edge="image", alpha=self.cfg.edge_aware_alpha).mean()
        return fn(flow, im1_scaled, edge="full_seg", full_seg=kw["full_seg"]).mean()

    def _image_pyramid(self, im, sizes):
        """{(h, w): F.interpolate(im, (h, w), mode="area")} for the loss scales,
        from one HIP pass (ops.area_pyramid, bit-exact) when the sizes are the
        exact halvings it computes; None otherwise (torch per scale)."""
        if not (self.fused and im.is_cuda):
            return None
        H, W = im.shape[-2:]
        want = {(H >> s, W >> s) for s in range(4)}
        if H % 8 or W % 8 or not set(sizes) <= want:
            return None
        from . import ops

        return dict(zip([(H >> s, W >> s) for s in range(4)], [im] + ops.area_pyramid(im)))

    def loss_one_pair(self, pyramid_flows, im1_origin, im2_origin, occ_aware=True, **kw):
        c = self.cfg
        dev = pyramid_flows[0].device
        sizes = [tuple(f.shape[-2:]) for i, f in enumerate(pyramid_flows) if c.w_ph_scales[i] > 0]
        pyr1 = self._image_pyramid(im1_origin, sizes)
        pyr2 = self._image_pyramid(im2_origin, sizes) if pyr1 is not None else None
        top = pyramid_flows[0]
        scale = min(*top.shape[-2:])
        vis = None
        if c.occ_from_back and self.lib_occ and top.is_cuda:
            # both masks from one HIP call (ops.occ_vis_pair): vis[0] = vis1, vis[1] = vis2
            from . import ops

            vis = ops.occ_vis_pair(top, th=0.2)
            vis1, vis2 = vis[0], vis[1]
        elif c.occ_from_back:
            vis1 = 1 - self.occ_backward(top[:, 2:], th=0.2)
            vis2 = 1 - self.occ_backward(top[:, :2], th=0.2)
        else:
            vis1 = 1 - self.occ_bidir(top[:, :2], top[:, 2:])
            vis2 = 1 - self.occ_bidir(top[:, 2:], top[:, :2])
        vis1_pyr, vis2_pyr = [vis1], [vis2]
        for i, f in enumerate(pyramid_flows[1:5], start=1):
            # (the reference also resizes the masks of scales it does not use;
            # only scales with a photometric weight read them)
            if occ_aware and c.w_ph_scales[i] <= 0:
                vis1_pyr.append(None)
                vis2_pyr.append(None)
                continue
            hw = tuple(f.shape[-2:])
            if vis is not None:  # both directions in one nearest resize
                B, _, H, W = top.shape
                v = F.interpolate(vis.view(2 * B, 1, H, W), hw, mode="nearest").view(2, B, 1, *hw)
                vis1_pyr.append(v[0])
                vis2_pyr.append(v[1])
            else:
                vis1_pyr.append(F.interpolate(vis1, hw, mode="nearest"))
                vis2_pyr.append(F.interpolate(vis2, hw, mode="nearest"))

        zero = torch.zeros((), dtype=torch.float32, device=dev)  # a fill, not an H2D copy (graph-capturable)
        # with_bk on the library's kernels: every weighted scale's photometric
        # pair in ONE launch (photometric_loss_pyramid; the per-scale results,
        # the small scales filling the chip's tail)
        pyr_losses = {}
        scales = [i for i, f in enumerate(pyramid_flows) if c.w_ph_scales[i] > 0]
        if (PHOTO_PYRAMID and c.with_bk and pyr1 is not None and 1 < len(scales) <= 4 and occ_aware
                and all(self._fused_photometric(pyramid_flows[i]) for i in scales)):
            from .photometric import photometric_loss_pyramid

            hws = [tuple(pyramid_flows[i].shape[-2:]) for i in scales]
            lp = photometric_loss_pyramid([pyramid_flows[i] for i in scales], [pyr1[hw] for hw in hws],
                                          [pyr2[hw] for hw in hws], [vis1_pyr[i] for i in scales],
                                          [vis2_pyr[i] for i in scales], c.warp_pad, c.w_l1, c.w_ssim)
            pyr_losses = {i: (lp[k, 0] + lp[k, 1]) / 2.0 for k, i in enumerate(scales)}
        warp_losses, smooth_losses = [], []
        for i, flow in enumerate(pyramid_flows):
            b, _, h, w = flow.size()
            im1_s = im2_s = None
            if i in pyr_losses:
                warp_losses.append(pyr_losses[i])
                if pyr1 is not None:
                    im1_s, im2_s = pyr1[(h, w)], pyr2[(h, w)]
            elif c.w_ph_scales[i] > 0:
                if pyr1 is not None:  # F.interpolate(im, (h, w), mode="area") from the HIP pyramid
                    im1_s, im2_s = pyr1[(h, w)], pyr2[(h, w)]
                else:
                    im1_s = F.interpolate(im1_origin, (h, w), mode="area")
                    im2_s = F.interpolate(im2_origin, (h, w), mode="area")
                if occ_aware:
                    m1, m2 = vis1_pyr[i], vis2_pyr[i]
                else:
                    m1 = torch.ones((b, 1, h, w), dtype=torch.float32, device=dev)
                    m2 = torch.ones((b, 1, h, w), dtype=torch.float32, device=dev)
                if self._fused_photometric(flow):
                    from .photometric import photometric_loss, photometric_loss_pair

                    if c.with_bk:  # both directions in one launch
                        lp = photometric_loss_pair(flow, im1_s, im2_s, m1, m2, c.warp_pad, c.w_l1, c.w_ssim)
                        lw = (lp[0] + lp[1]) / 2.0
                    else:
                        lw = photometric_loss(flow[:, :2], im2_s, im1_s, m1, c.warp_pad, c.w_l1, c.w_ssim)
                else:
                    im1_rec = self.warp(im2_s, flow[:, :2], pad=c.warp_pad)
                    im2_rec = self.warp(im1_s, flow[:, 2:], pad=c.warp_pad)
                    lw = self.loss_photomatric(im1_s, im1_rec, m1)
                    if c.with_bk:
                        lw = (lw + self.loss_photomatric(im2_s, im2_rec, m2)) / 2.0
                warp_losses.append(lw)
            else:
                warp_losses.append(zero)

            if i == 0 and c.w_sm > 0:
                if c.smooth_type == "homography":
                    raise NotImplementedError("homography smoothness needs OpenCV RANSAC (not on the hot path)")
                if im1_s is None:
                    im1_s = F.interpolate(im1_origin, (h, w), mode="area")
                    im2_s = F.interpolate(im2_origin, (h, w), mode="area")
                ls = self.loss_smooth(flow[:, :2] / scale, im1_s, full_seg=kw.get("full_seg1"))
                if c.with_bk:
                    ls = (ls + self.loss_smooth(flow[:, 2:] / scale, im2_s, full_seg=kw.get("full_seg2"))) / 2.0
                smooth_losses.append(ls)
            else:
                smooth_losses.append(zero)

        l_ph = sum(l * wt for l, wt in zip(warp_losses, c.w_ph_scales))
        l_sm = sum(smooth_losses)
        loss = l_ph + c.w_sm * l_sm
        return loss, l_ph, l_sm, top[:, :2].norm(dim=1).mean(), vis1_pyr[0], vis2_pyr[0]

    def forward(self, pyramid_flows, img1, img2, occ_aware=True, **kw):
        loss, l_ph, l_sm, fmean, v1, v2 = self.loss_one_pair(pyramid_flows, img1, img2, occ_aware=occ_aware, **kw)
        return loss[None], l_ph[None], l_sm[None], fmean[None], v1, v2
