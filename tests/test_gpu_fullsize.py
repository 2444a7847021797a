"""The dominant shapes pinned directly against the CPU oracle (VERDICT r02
"pin the dominant shapes"):

* the loss's full-resolution photometric pair (both with_bk directions,
  8x3x256x832, flow_loss.py:130-148) -- the kernel that sets the roofline
  site -- against the oracle composition (oracle flow_warp + the torch L1/SSIM
  of loss_photomatric), loss values and flow gradients (sums, abs-sums and
  4096 sampled elements);
* one full-size KITTI training step (B=1, 832x256, kitti_base) against the
  same step on the CPU with the oracle ops, as smoke_step does at 64x128:
  loss, the five output flows, per-parameter gradient sums.

Tolerances are the photometric tests' (loss rtol 2e-5; gradient atol 2e-4 x
max|g| + rtol 1e-3) and the reference-capture test's (flows atol 1e-4 /
rtol 1e-3, loss rtol 1e-4, gradient sums within 2e-3 of the abs-sum): the
convolutions run on MIOpen here and on the CPU in the oracle step.
"""
import numpy as np
import pytest
import torch

from oracle import hashrng
from oracle.torch_ref import oracle_flow_warp

pytestmark = pytest.mark.gpu


def _smooth_flow(B, H, W, seed, amp):
    """[B,4,H,W]: two low-frequency sinusoids per component (+-amp px) plus
    a little per-pixel noise, as a mid-training flow field looks."""
    yy = np.linspace(0, 2 * np.pi, H, dtype=np.float32)[:, None]
    xx = np.linspace(0, 2 * np.pi, W, dtype=np.float32)[None, :]
    ph = hashrng.uniform((B, 4), seed) * np.float32(2 * np.pi)
    f = np.empty((B, 4, H, W), np.float32)
    for b in range(B):
        for k in range(4):
            f[b, k] = amp * 0.5 * (np.sin(2 * xx + ph[b, k]) + np.cos(3 * yy - ph[b, k]))
    f += hashrng.symmetric((B, 4, H, W), seed + 1, 0.25)
    return torch.from_numpy(f)


def _ref_loss(flow, src, tgt, mask, pad):
    from unsamflow_amd.config import AttrDict
    from unsamflow_amd.flow_loss import unFlowLoss

    lf = unFlowLoss(AttrDict.wrap(dict(w_l1=0.15, w_ssim=0.85, w_ternary=0.0)), warp_fn=oracle_flow_warp)
    return lf.loss_photomatric(tgt, oracle_flow_warp(src, flow, pad=pad), mask)


def test_photometric_pair_full_kitti_vs_oracle(hip_device):
    from unsamflow_amd.photometric import photometric_loss_pair

    B, C, H, W = 8, 3, 256, 832
    im1 = torch.from_numpy(hashrng.uniform((B, C, H, W), 501))
    im2 = torch.from_numpy(hashrng.uniform((B, C, H, W), 502))
    flow = _smooth_flow(B, H, W, 503, 3.0)
    m1 = (torch.from_numpy(hashrng.uniform((B, 1, H, W), 505)) > 0.15).float()
    m2 = (torch.from_numpy(hashrng.uniform((B, 1, H, W), 506)) > 0.25).float()
    d = hip_device

    fp = flow.to(d).requires_grad_(True)
    lp = photometric_loss_pair(fp, im1.to(d), im2.to(d), m1.to(d), m2.to(d), "border", 0.15, 0.85)
    (lp[0] * 0.7 + lp[1] * 1.3).backward()
    g = fp.grad.cpu().numpy()

    fr = flow.clone().requires_grad_(True)
    r0 = _ref_loss(fr[:, :2], im2, im1, m1, "border")
    r1 = _ref_loss(fr[:, 2:], im1, im2, m2, "border")
    (r0 * 0.7 + r1 * 1.3).backward()
    gref = fr.grad.numpy()

    np.testing.assert_allclose(lp.detach().cpu().numpy(), [float(r0), float(r1)], rtol=2e-5, atol=0)
    gmax = float(np.abs(gref).max())
    for k in range(4):  # per flow channel: sum and abs-sum within 1e-3 of the abs-sum
        a, r = g[:, k].astype(np.float64), gref[:, k].astype(np.float64)
        assert abs(a.sum() - r.sum()) <= 1e-3 * np.abs(r).sum(), k
        np.testing.assert_allclose(np.abs(a).sum(), np.abs(r).sum(), rtol=1e-3)
    idx = (hashrng.uniform((4096,), 507) * g.size).astype(np.int64)
    np.testing.assert_allclose(g.reshape(-1)[idx], gref.reshape(-1)[idx], rtol=1e-3, atol=2e-4 * gmax)


def test_train_step_full_kitti_b1_vs_oracle(hip_device):
    """smoke_step's check at the real frame size: B=1, 832x256."""
    from oracle.hashrng import hash_init_, uniform
    from oracle.torch_ref import OracleCorrelation, oracle_occu_mask_backward
    from unsamflow_amd.config import kitti_base
    from unsamflow_amd.harness import TrainStep

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    gpu = TrainStep(kitti_base(), hip_device)
    cpu = TrainStep(kitti_base(), "cpu", corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                    occ_backward_fn=oracle_occu_mask_backward)
    hash_init_(gpu.module, seed=1)
    hash_init_(cpu.module, seed=1)
    im1 = torch.from_numpy(uniform((1, 3, 256, 832), 21))
    im2 = torch.from_numpy(uniform((1, 3, 256, 832), 22))
    lg, fg = gpu.forward_loss(im1.to(hip_device), im2.to(hip_device))
    lc, fc = cpu.forward_loss(im1, im2)
    lg.backward()
    lc.backward()
    torch.cuda.synchronize(hip_device)
    assert abs(lg.item() - lc.item()) <= 1e-4 * abs(lc.item()) + 1e-6, (lg.item(), lc.item())
    for a, b in zip(fg, fc):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().numpy(), atol=1e-4, rtol=1e-3)
    for (n, pg), pc in zip(gpu.module.named_parameters(), cpu.module.parameters()):
        ga = float(pc.grad.double().abs().sum())
        assert abs(float(pg.grad.double().sum()) - float(pc.grad.double().sum())) <= 2e-3 * ga + 1e-8, n
        assert abs(float(pg.grad.double().abs().sum()) - ga) <= 2e-3 * ga + 1e-8, n


def test_train_step_full_sintel_mf_b1_vs_oracle(hip_device):
    """SURVEY config 5 per GPU at its real size: Sintel 1024x448, the mask-feature
    branch on (configs/sintel_aug+hg+mf.json:3-6: add_mask_corr, aggregation
    "concat"; pwclite.py:317-361), B=1, K=32 piecewise-constant SAM segments --
    the HIP step against the CPU oracle step (loss, flows, gradient sums), with
    the same tolerances as the KITTI step above."""
    from oracle.hashrng import hash_init_, uniform
    from oracle.torch_ref import OracleCorrelation, oracle_occu_mask_backward
    from unsamflow_amd.config import sintel_mf
    from unsamflow_amd.harness import TrainStep, synthetic_pair

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = sintel_mf()
    assert cfg.model.add_mask_corr
    gpu = TrainStep(cfg, hip_device)
    cpu = TrainStep(cfg, "cpu", corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                    occ_backward_fn=oracle_occu_mask_backward)
    hash_init_(gpu.module, seed=3)
    hash_init_(cpu.module, seed=3)
    H, W = 448, 1024
    im1 = torch.from_numpy(uniform((1, 3, H, W), 31))
    im2 = torch.from_numpy(uniform((1, 3, H, W), 32))
    _, _, s1, s2 = synthetic_pair(1, H, W, "cpu", seed=33, with_seg=True, n_seg=32)
    d = hip_device
    lg, fg = gpu.forward_loss(im1.to(d), im2.to(d), s1.to(d), s2.to(d))
    lc, fc = cpu.forward_loss(im1, im2, s1, s2)
    lg.backward()
    lc.backward()
    torch.cuda.synchronize(d)
    assert abs(lg.item() - lc.item()) <= 1e-4 * abs(lc.item()) + 1e-6, (lg.item(), lc.item())
    assert len(fg) == len(fc) == 5
    for a, b in zip(fg, fc):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().numpy(), atol=1e-4, rtol=1e-3)
    n_mask = 0
    for (n, pg), pc in zip(gpu.module.named_parameters(), cpu.module.parameters()):
        n_mask += "mask" in n
        ga = float(pc.grad.double().abs().sum())
        assert abs(float(pg.grad.double().sum()) - float(pc.grad.double().sum())) <= 2e-3 * ga + 1e-8, n
        assert abs(float(pg.grad.double().abs().sum()) - ga) <= 2e-3 * ga + 1e-8, n
    assert n_mask > 0  # the mask-feature branch's own parameters took part
