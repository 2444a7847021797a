"""Fused photometric loss (unsamflow_amd.photometric, csrc/photo.hip) vs the
reference composition on the CPU: oracle flow_warp (grid_sample) + the torch
L1/SSIM of loss_photomatric (flow_loss.py:33-50, loss_blocks.py:53-72), fp32.
Loss value: rtol 2e-5. grad_flow: atol 2e-4 x max|grad| + rtol 1e-3 (the
backward sums the 9 SSIM windows and the channels in another order)."""
import numpy as np
import pytest
import torch

from oracle import hashrng
from oracle.torch_ref import oracle_flow_warp

pytestmark = pytest.mark.gpu


def _ref_loss(flow, src, tgt, mask, pad, w_l1, w_ssim):
    from unsamflow_amd.config import AttrDict
    from unsamflow_amd.flow_loss import unFlowLoss

    cfg = AttrDict.wrap(dict(w_l1=w_l1, w_ssim=w_ssim, w_ternary=0.0))
    lf = unFlowLoss(cfg, warp_fn=oracle_flow_warp)
    rec = oracle_flow_warp(src, flow, pad=pad)
    return lf.loss_photomatric(tgt, rec, mask)


CASES = [
    # (B, C, H, W, flow scale, mask kind, pad)
    (2, 3, 24, 40, 2.0, "rand", "border"),
    (2, 3, 17, 29, 6.0, "ones", "border"),
    (1, 3, 3, 5, 1.0, "rand", "border"),
    (2, 3, 33, 47, 3.0, "rand", "zeros"),
    (2, 1, 20, 36, 2.0, "rand", "border"),
    (2, 2, 21, 70, 2.0, "rand", "border"),  # the C == 2 instantiation (advisor r03)
    (8, 3, 64, 208, 4.0, "rand", "border"),
]


@pytest.mark.parametrize("B,C,H,W,scale,mkind,pad", CASES)
def test_photometric_loss_matches_reference_composition(hip_device, B, C, H, W, scale, mkind, pad):
    from unsamflow_amd.photometric import photometric_loss

    seed = 100 + H + W
    src = torch.from_numpy(hashrng.uniform((B, C, H, W), seed))
    tgt = torch.from_numpy(hashrng.uniform((B, C, H, W), seed + 1))
    flow_full = torch.from_numpy(hashrng.symmetric((B, 4, H, W), seed + 2, scale))
    if mkind == "ones":
        mask = torch.ones(B, 1, H, W)
    else:
        mask = (torch.from_numpy(hashrng.uniform((B, 1, H, W), seed + 3)) > 0.2).float()

    fr = flow_full.clone().requires_grad_(True)
    ref = _ref_loss(fr[:, :2], src, tgt, mask, pad, 0.15, 0.85)
    ref.backward()
    gref = fr.grad[:, :2].numpy()

    fd = flow_full.to(hip_device).requires_grad_(True)
    out = photometric_loss(fd[:, :2], src.to(hip_device), tgt.to(hip_device), mask.to(hip_device), pad,
                           0.15, 0.85)
    out.backward()
    g = fd.grad[:, :2].cpu().numpy()
    assert float(fd.grad[:, 2:].abs().max()) == 0.0
    np.testing.assert_allclose(float(out), float(ref), rtol=2e-5, atol=0)
    np.testing.assert_allclose(g, gref, rtol=1e-3, atol=2e-4 * float(np.abs(gref).max()))


def test_photometric_loss_in_unflowloss_matches_torch_path(hip_device):
    """unFlowLoss with the fused op == unFlowLoss with the library warp + torch
    L1/SSIM (fused_photometric=False), value and flow gradients, at the KITTI
    loss pyramid (4 scales, B=2, 256x832 top)."""
    from unsamflow_amd.config import kitti_base
    from unsamflow_amd.flow_loss import unFlowLoss

    cfg = kitti_base().loss
    B = 2
    img1 = torch.from_numpy(hashrng.uniform((B, 3, 256, 832), 11)).to(hip_device)
    img2 = torch.from_numpy(hashrng.uniform((B, 3, 256, 832), 12)).to(hip_device)
    flows = [torch.from_numpy(hashrng.symmetric((B, 4, 256 >> i, 832 >> i), 20 + i, 3.0 / (1 << i)))
             for i in range(5)]
    res = []
    for fused in (True, False):
        fl = [f.to(hip_device).requires_grad_(True) for f in flows]
        loss = unFlowLoss(cfg, fused_photometric=fused)(fl, img1, img2)[0].sum()
        loss.backward()
        res.append((float(loss), [None if f.grad is None else f.grad.cpu().numpy() for f in fl]))
    (lf, gf), (lt, gt) = res
    np.testing.assert_allclose(lf, lt, rtol=2e-5)
    for a, b in zip(gf, gt):  # the 5th level has photometric weight 0 (no gradient at all)
        assert (a is None) == (b is None)
        if a is not None:
            np.testing.assert_allclose(a, b, rtol=1e-3, atol=2e-4 * max(float(np.abs(b).max()), 1e-12))


PAIR_CASES = [
    (2, 3, 24, 40, 2.0, "border"),
    (1, 3, 3, 5, 1.0, "border"),
    (2, 1, 33, 47, 3.0, "zeros"),
    (2, 2, 19, 130, 2.0, "zeros"),
    (8, 3, 64, 208, 4.0, "border"),
]


@pytest.mark.parametrize("B,C,H,W,scale,pad", PAIR_CASES)
def test_photometric_pair_matches_reference_and_single_directions(hip_device, B, C, H, W, scale, pad):
    """Both with_bk directions in one launch == the two single-direction calls
    (bit-identical: same kernel body per direction) and == the reference
    composition of each direction (flow_loss.py:130-131, 143-148)."""
    from unsamflow_amd.photometric import photometric_loss, photometric_loss_pair

    seed = 300 + H + W
    im1 = torch.from_numpy(hashrng.uniform((B, C, H, W), seed))
    im2 = torch.from_numpy(hashrng.uniform((B, C, H, W), seed + 1))
    flow = torch.from_numpy(hashrng.symmetric((B, 4, H, W), seed + 2, scale))
    m1 = (torch.from_numpy(hashrng.uniform((B, 1, H, W), seed + 3)) > 0.2).float()
    m2 = (torch.from_numpy(hashrng.uniform((B, 1, H, W), seed + 4)) > 0.3).float()
    d = hip_device

    fp = flow.to(d).requires_grad_(True)
    lp = photometric_loss_pair(fp, im1.to(d), im2.to(d), m1.to(d), m2.to(d), pad, 0.15, 0.85)
    (lp[0] * 0.7 + lp[1] * 1.3).backward()

    fs = flow.to(d).requires_grad_(True)
    l0 = photometric_loss(fs[:, :2], im2.to(d), im1.to(d), m1.to(d), pad, 0.15, 0.85)
    l1 = photometric_loss(fs[:, 2:], im1.to(d), im2.to(d), m2.to(d), pad, 0.15, 0.85)
    (l0 * 0.7 + l1 * 1.3).backward()
    assert torch.equal(lp.detach().cpu(), torch.stack([l0, l1]).detach().cpu())
    assert torch.equal(fp.grad.cpu(), fs.grad.cpu())

    fr = flow.clone().requires_grad_(True)
    r0 = _ref_loss(fr[:, :2], im2, im1, m1, pad, 0.15, 0.85)
    r1 = _ref_loss(fr[:, 2:], im1, im2, m2, pad, 0.15, 0.85)
    (r0 * 0.7 + r1 * 1.3).backward()
    np.testing.assert_allclose(lp.detach().cpu().numpy(), [float(r0), float(r1)], rtol=2e-5, atol=0)
    gref = fr.grad.numpy()
    np.testing.assert_allclose(fp.grad.cpu().numpy(), gref, rtol=1e-3, atol=2e-4 * float(np.abs(gref).max()))


def test_photometric_forward_only_matches_grad_forward(hip_device):
    """The no-grad instantiation (no basis) computes the same loss value (up to
    FMA contraction choices of the two instantiations)."""
    from unsamflow_amd import ops

    B, C, H, W = 2, 3, 40, 72
    src = torch.from_numpy(hashrng.uniform((B, C, H, W), 7)).to(hip_device)
    tgt = torch.from_numpy(hashrng.uniform((B, C, H, W), 8)).to(hip_device)
    flow = torch.from_numpy(hashrng.symmetric((B, 2, H, W), 9, 3.0)).to(hip_device)
    mask = (torch.from_numpy(hashrng.uniform((B, 1, H, W), 10)) > 0.2).float().to(hip_device)
    a, basis = ops.photo_loss_forward(src, tgt, mask, flow, "border", need_grad=True)
    b, none = ops.photo_loss_forward(src, tgt, mask, flow, "border", need_grad=False)
    assert none is None and basis.shape == (B, 4, H, W)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=0)


@pytest.mark.parametrize("pad", ["border", "zeros"])
@pytest.mark.parametrize("B,C,sizes", [(8, 3, [(256, 832), (128, 416), (64, 208), (32, 104)]),
                                        (2, 3, [(33, 47), (17, 24)]), (2, 1, [(40, 64), (20, 32), (10, 16)])])
def test_photometric_pyramid_equals_per_scale_pairs(hip_device, B, C, sizes, pad):
    """photometric_loss_pyramid (usf_photo_loss_pyramid_{fwd,bwd}_f32: every
    loss scale in one forward launch and one backward launch) gives the
    per-scale photometric_loss_pair results bit for bit -- losses and each
    scale's flow gradient -- at the KITTI loss scales (B=8, 832x256 down to
    104x32) and odd sizes; the per-scale form is itself checked against the
    reference composition above."""
    from unsamflow_amd.photometric import photometric_loss_pair, photometric_loss_pyramid

    flows, i1, i2, m1, m2 = [], [], [], [], []
    for k, (H, W) in enumerate(sizes):
        flows.append(torch.from_numpy(hashrng.symmetric((B, 4, H, W), 950 + k, 3.0)).to(hip_device))
        i1.append(torch.from_numpy(hashrng.uniform((B, C, H, W), 960 + k)).to(hip_device))
        i2.append(torch.from_numpy(hashrng.uniform((B, C, H, W), 970 + k)).to(hip_device))
        m1.append((torch.from_numpy(hashrng.uniform((B, 1, H, W), 980 + k)) > 0.2).float().to(hip_device))
        m2.append((torch.from_numpy(hashrng.uniform((B, 1, H, W), 990 + k)) > 0.2).float().to(hip_device))
    fa = [f.clone().requires_grad_(True) for f in flows]
    fb = [f.clone().requires_grad_(True) for f in flows]
    lp = photometric_loss_pyramid(fa, i1, i2, m1, m2, pad)
    ref = torch.stack([photometric_loss_pair(f, a, b, x, y, pad) for f, a, b, x, y in zip(fb, i1, i2, m1, m2)])
    assert torch.equal(lp, ref)
    wts = torch.arange(1, 2 * len(sizes) + 1, device=hip_device, dtype=torch.float32).view(-1, 2)
    (lp * wts).sum().backward()
    (ref * wts).sum().backward()
    for a, b in zip(fa, fb):
        assert torch.equal(a.grad, b.grad)
