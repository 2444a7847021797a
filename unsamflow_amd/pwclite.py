"""PWCLite — the caller of the hot path (models/pwclite.py), rebuilt here so the
benchmark can run the reference's training step on the GPU box.

Module tree, parameter names/shapes and the forward computation follow
``models/pwclite.py`` so a reference ``state_dict`` loads unchanged:

* ``feature_pyramid_extractor`` — 6 x [3x3 s2 conv, 3x3 conv] + LeakyReLU(0.1),
  optional adjacency-map stem (pwclite.py:42-76);
* decoder (pwclite.py:278-385): per level, bilinear x2 flow upsampling
  (align_corners), **flow_warp** of x2 by the flow (:302), **Correlation**
  d=4 (:307) + in-place LeakyReLU (:308), 1x1 feature conv, optional
  mask-feature correlation branch (:317-361), FlowEstimatorReduce/Dense,
  ContextNetwork residual, convex (learned) or bilinear x4 upsampling;
* ``forward(img1, img2, full_seg1=None, full_seg2=None, with_bk=False)``
  returns ``{"flows_12": [...], "flows_21": [...]}`` (:387-434).

The correlation and warp are the HIP drop-ins by default. ``corr_module`` /
``warp_fn`` can be injected — the CPU tests inject the oracle restatement;
the product path never falls back to anything.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv_block(cin: int, cout: int, k: int = 3, stride: int = 1, dilation: int = 1, relu: bool = True) -> nn.Sequential:
    """Conv2d ('same' padding for odd k) [+ LeakyReLU(0.1, inplace)] — key layout ``.0.weight``."""
    layers = [nn.Conv2d(cin, cout, k, stride=stride, dilation=dilation, padding=((k - 1) * dilation) // 2, bias=True)]
    if relu:
        layers.append(nn.LeakyReLU(0.1, inplace=True))
    return nn.Sequential(*layers)


def full_segs_to_adj_maps(full_segs: torch.Tensor, win_size: int = 9, pad_mode: str = "replicate") -> torch.Tensor:
    """[B,1,H,W] segment ids -> [B,win^2,H,W] same-segment indicator (input_transforms.py:35-49)."""
    r = (win_size - 1) // 2
    b, _, h, w = full_segs.shape
    nb = F.unfold(F.pad(full_segs, (r, r, r, r), mode=pad_mode), [win_size, win_size])
    return (full_segs == nb.reshape(b, win_size * win_size, h, w)).float()


class FeatureExtractor(nn.Module):
    def __init__(self, num_chs, input_adj_map: bool = False):
        super().__init__()
        self.num_chs = num_chs
        self.adj_map_net = None
        if input_adj_map:
            self.adj_map_net = nn.Sequential(
                conv_block(81, 32, k=1), conv_block(32, 32, stride=2), conv_block(32, 32),
                conv_block(32, 32, stride=2), conv_block(32, 32),
            )
        self.convs = nn.ModuleList()
        for lvl in range(len(num_chs) - 1):
            cin = num_chs[lvl] + (32 if input_adj_map and lvl == 2 else 0)
            cout = num_chs[lvl + 1]
            self.convs.append(nn.Sequential(conv_block(cin, cout, stride=2), conv_block(cout, cout)))

    def forward(self, x, adj_map=None):
        adj = self.adj_map_net(adj_map) if self.adj_map_net is not None else None
        pyramid = [x]
        for lvl, block in enumerate(self.convs):
            if adj is not None and lvl == 2:
                x = torch.cat((x, adj), dim=1)
            x = block(x)
            pyramid.append(x)
        return pyramid[::-1]  # coarsest first


class FlowEstimatorDense(nn.Module):
    def __init__(self, ch_in: int):
        super().__init__()
        widths = [128, 128, 96, 64, 32]
        acc = ch_in
        for i, w in enumerate(widths, 1):
            setattr(self, f"conv{i}", conv_block(acc, w))
            acc += w
        self.feat_dim = acc
        self.conv_last = conv_block(acc, 2, relu=False)

    def forward(self, x):
        for i in range(1, 6):
            x = torch.cat([getattr(self, f"conv{i}")(x), x], dim=1)
        return x, self.conv_last(x)


class FlowEstimatorReduce(nn.Module):
    """Dense estimator with each conv seeing only the two previous outputs."""

    def __init__(self, ch_in: int):
        super().__init__()
        self.conv1 = conv_block(ch_in, 128)
        self.conv2 = conv_block(128, 128)
        self.conv3 = conv_block(256, 96)
        self.conv4 = conv_block(224, 64)
        self.conv5 = conv_block(160, 32)
        self.feat_dim = 32
        self.predict_flow = conv_block(96, 2, relu=False)

    def forward(self, x):
        a = self.conv1(x)
        b = self.conv2(a)
        c = self.conv3(torch.cat([a, b], 1))
        d = self.conv4(torch.cat([b, c], 1))
        e = self.conv5(torch.cat([c, d], 1))
        return e, self.predict_flow(torch.cat([d, e], 1))


class ContextNetwork(nn.Module):
    def __init__(self, ch_in: int):
        super().__init__()
        self.convs = nn.Sequential(*[conv_block(ci, co, 3, 1, dil) for ci, co, dil in
                                     ((ch_in, 128, 1), (128, 128, 2), (128, 128, 4), (128, 96, 8))])
        self.flow_head = nn.Sequential(conv_block(96, 64, 3, 1, 16), conv_block(64, 32, 3, 1, 1),
                                       conv_block(32, 2, relu=False))

    def forward(self, x):
        feat = self.convs(x)
        return self.flow_head(feat), feat


class UpFlowNetwork(nn.Module):
    """Convex x4 upsampler (RAFT-style mask over the 3x3 neighbourhood)."""

    def __init__(self, ch_in: int = 96, scale_factor: int = 4):
        super().__init__()
        self.scale = scale_factor
        self.fused = False  # PWCLite turns on the HIP op (csrc/convex.hip) with its own corr/warp
        self.convs = nn.Sequential(conv_block(ch_in, 128, 3, 1, 1), conv_block(128, scale_factor ** 2 * 9, 3, 1, 1))

    def upsample_flow(self, flow, mask):
        N, _, H, W = flow.shape
        s = self.scale
        weights = torch.softmax(mask.view(N, 1, 9, s, s, H, W), dim=2)
        patches = F.unfold(s * flow, [3, 3], padding=1).view(N, 2, 9, 1, 1, H, W)
        up = torch.sum(weights * patches, dim=2)  # N,2,s,s,H,W
        return up.permute(0, 1, 4, 2, 5, 3).reshape(N, 2, s * H, s * W)

    def mask(self, feat):
        """The convs' raw upsampling mask (the 0.25 scale is applied by the op)."""
        return self.convs(feat)

    def forward(self, flow, feat):
        if self.fused and flow.is_cuda:
            from .upsample import convex_upsample

            return convex_upsample(flow, self.convs(feat), self.scale, 0.25)
        return self.upsample_flow(flow, 0.25 * self.convs(feat))


def _default_corr():
    from .correlation import Correlation

    return Correlation(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=1)


# the decoder's x2 flow upsampling and warp of x2 as one launch (upsample.upsample_warp)
FUSED_UP_WARP = True


def _default_warp():
    from .warp_utils import flow_warp

    return flow_warp


class PWCLite(nn.Module):
    def __init__(self, cfg, corr_module: nn.Module | None = None, warp_fn: Callable | None = None):
        super().__init__()
        for key in ("input_adj_map", "input_boundary", "add_mask_corr"):
            if key not in cfg:
                cfg[key] = False
        self.cfg = cfg
        self.search_range = 4
        self.num_chs = [3, 16, 32, 64, 96, 128, 192]
        if cfg.input_boundary:
            self.num_chs[0] += 2
        self.output_level = 4
        # with_bk as one pass at batch 2B (_forward_batched); False: the reference's two passes
        self.batch_directions = True
        self.num_levels = 7
        self.leakyRELU = nn.LeakyReLU(0.1, inplace=True)
        self.warp = warp_fn if warp_fn is not None else _default_warp()

        self.feature_pyramid_extractor = FeatureExtractor(self.num_chs, input_adj_map=cfg.input_adj_map)
        self.corr = corr_module if corr_module is not None else _default_corr()
        # the fused corr + LeakyReLU + concat op (corr_cat.py) stands in for the
        # library's own Correlation module only; an injected module keeps the
        # reference composition
        self.fused_corr_cat = corr_module is None
        self.dim_corr = (2 * self.search_range + 1) ** 2
        self.num_ch_in = 32 + (2 if cfg.add_mask_corr else 1) * self.dim_corr + 2
        self.flow_estimators = (FlowEstimatorReduce if cfg.reduce_dense else FlowEstimatorDense)(self.num_ch_in)
        self.context_networks = ContextNetwork(self.flow_estimators.feat_dim + 2)
        self.output_flow_upsampler = UpFlowNetwork(ch_in=96, scale_factor=4) if cfg.learned_upsampler else None
        if self.output_flow_upsampler is not None:
            self.output_flow_upsampler.fused = self.fused_corr_cat
        # 1x1 projections of the decoder levels' features (192, 128, 96, 64, 32 channels)
        level_chs = self.num_chs[::-1][:5]
        self.conv_1x1 = nn.ModuleList([conv_block(c, 32, k=1) for c in level_chs])
        if cfg.add_mask_corr:
            self.conv_1x1_mask = nn.ModuleList([conv_block(c, 32, k=1) for c in level_chs])
            if cfg.aggregation_type == "residual":
                self.mask_aggregation = conv_block(32, 32, k=1)
            elif cfg.aggregation_type == "concat":
                self.mask_aggregation = conv_block(64, 32, k=1)

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    # -- mask-feature branch (pwclite.py:317-357) ------------------------------
    def _mask_feature(self, x, full_seg, level):
        proj = self.conv_1x1_mask[level](x)
        seg = F.interpolate(full_seg, x.shape[-2:], mode="nearest").long()
        onehot = F.one_hot(seg)  # [B,1,h,w,K]
        pooled = torch.amax(onehot * proj[..., None], dim=(2, 3))  # [B,32,K]: per-segment max
        spread = (onehot * pooled[:, :, None, None, :]).sum(dim=-1)  # back to pixels
        if self.cfg.aggregation_type == "residual":
            return proj + self.mask_aggregation(spread)
        if self.cfg.aggregation_type == "concat":
            return self.mask_aggregation(torch.cat((proj, spread), dim=1))
        raise NotImplementedError(self.cfg.aggregation_type)

    def _upsample(self, flow, k):
        """F.interpolate(flow * k, scale_factor=k, bilinear, align_corners=True) (:299-301);
        the HIP op (upsample.py) next to the library's own corr/warp."""
        if self.fused_corr_cat and flow.is_cuda:
            from .upsample import upsample_flow

            return upsample_flow(flow, k)
        return F.interpolate(flow * k, scale_factor=k, mode="bilinear", align_corners=True)

    def _fused_up_warp(self, flow):
        """The library's own upsampling and warp on a ROCm device (not an injected warp)."""
        from .warp_utils import flow_warp

        return FUSED_UP_WARP and self.fused_corr_cat and flow.is_cuda and self.warp is flow_warp

    def decoder(self, x1_pyramid, x2_pyramid, full_seg1=None, full_seg2=None):
        flows, deferred = [], []
        B, _, h0, w0 = x1_pyramid[0].size()
        flow = torch.zeros(B, 2, h0, w0, dtype=x1_pyramid[0].dtype, device=x1_pyramid[0].device).float()
        for level, (x1, x2) in enumerate(zip(x1_pyramid, x2_pyramid)):
            if level > 0 and self._fused_up_warp(flow):
                # x2 upsampling and the warp of x2 in one launch (the same numbers)
                from .upsample import upsample_warp

                flow, x2_warp = upsample_warp(flow, x2)
            elif level > 0:
                flow = self._upsample(flow, 2)
                x2_warp = self.warp(x2, flow)
            else:
                x2_warp = x2
            pairs = [(x1, x2_warp)]
            if self.cfg.add_mask_corr:
                m1 = self._mask_feature(x1, full_seg1, level)
                m2 = self._mask_feature(x2, full_seg2, level)
                pairs.append((m1, self.warp(m2, flow)))
            extras = [self.conv_1x1[level](x1), flow]
            if self.fused_corr_cat and x1.is_cuda:
                # LeakyReLU + concat fused into the correlation kernels (corr_cat.py)
                from .corr_cat import corr_leaky_cat

                est_in = corr_leaky_cat(pairs, extras, self.search_range, 0.1)
            else:
                est_in = torch.cat([self.leakyRELU(self.corr(a, b)) for a, b in pairs] + extras, dim=1)
            x_intm, flow_res = self.flow_estimators(est_in)
            flow = flow + flow_res
            flow_fine, up_feat = self.context_networks(torch.cat([x_intm, flow], dim=1))
            flow = flow + flow_fine
            up = self.output_flow_upsampler
            if up is not None and up.fused and flow.is_cuda and up.scale == 4:
                # the upsampled flows feed only the loss: every level's convex
                # upsampling runs in one launch after the loop (the same numbers)
                deferred.append((flow, up.mask(up_feat)))
            elif up is not None:
                flows.append(up(flow, up_feat))
            else:
                flows.append(self._upsample(flow, 4))
            if level == self.output_level:
                break
        if deferred:  # finest level first: the largest level's blocks lead the grid
            from .upsample import convex_upsample_pyramid

            return convex_upsample_pyramid([f for f, _ in deferred[::-1]], [m for _, m in deferred[::-1]], 4, 0.25)
        return flows[::-1]

    @staticmethod
    def _seg_edges(full_seg):
        B, _, h, w = full_seg.shape
        ex = (full_seg[..., :, 1:] != full_seg[..., :, :-1]).float()
        ey = (full_seg[..., 1:, :] != full_seg[..., :-1, :]).float()
        ex = torch.cat((ex, ex.new_zeros(B, 1, h, 1)), dim=-1)
        ey = torch.cat((ey, ey.new_zeros(B, 1, 1, w)), dim=-2)
        return ex, ey

    def forward(self, img1, img2, full_seg1=None, full_seg2=None, with_bk=False):
        B = img1.shape[0]
        adj1 = adj2 = None
        if self.cfg.input_adj_map:
            adj = full_segs_to_adj_maps(torch.cat((full_seg1, full_seg2), dim=0))
            adj1, adj2 = adj[:B], adj[B:]
        if self.cfg.input_boundary:
            img1 = torch.cat((img1, *self._seg_edges(full_seg1)), dim=1)
            img2 = torch.cat((img2, *self._seg_edges(full_seg2)), dim=1)
        if with_bk and self.batch_directions:
            return self._forward_batched(img1, img2, full_seg1, full_seg2, adj1, adj2)
        feat1 = self.feature_pyramid_extractor(img1, adj1)
        feat2 = self.feature_pyramid_extractor(img2, adj2)
        res = {"flows_12": self.decoder(feat1, feat2, full_seg1, full_seg2)}
        if with_bk:
            res["flows_21"] = self.decoder(feat2, feat1, full_seg2, full_seg1)
        return res

    def _forward_batched(self, img1, img2, full_seg1, full_seg2, adj1, adj2):
        """with_bk as ONE pass at batch 2B: the reference runs the feature extractor
        per frame and the decoder per direction (pwclite.py:425-432), i.e. the same
        per-sample computation twice at batch B. Stacking [frame 1; frame 2] and
        [direction 12; direction 21] along the batch gives identical per-sample
        results with half the launches, each twice as large: the coarse levels'
        convolutions and the hot-path kernels at L0-L2 are latency-bound at B = 8
        and fill the 256 CUs better at 16. Only the weight-gradient sums over the
        batch change order."""
        B = img1.shape[0]
        adj = torch.cat((adj1, adj2), dim=0) if adj1 is not None else None
        feats = self.feature_pyramid_extractor(torch.cat((img1, img2), dim=0), adj)
        used = feats[: self.output_level + 1]
        swapped = [torch.cat((f[B:], f[:B]), dim=0) for f in used]
        seg_a = seg_b = None
        if full_seg1 is not None:
            seg_a = torch.cat((full_seg1, full_seg2), dim=0)
            seg_b = torch.cat((full_seg2, full_seg1), dim=0)
        flows = self.decoder(used, swapped, seg_a, seg_b)
        return {"flows_12": [f[:B] for f in flows], "flows_21": [f[B:] for f in flows]}
