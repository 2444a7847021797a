"""get_occu_mask_bidirection (utils/warp_utils.py:109-117) as one HIP kernel
(usf_occ_bidirection_f32) against the float32 numpy oracle
(oracle.warp.occu_mask_bidirection_np, pinned through the reference's own
zeros-mode warp goldens, tests/test_oracle_golden.py) and against the
composition the reference evaluates (HIP zeros-padded flow_warp + the
element-wise test in torch). Mask decisions must be equal except within
rounding of the threshold (|d|^2 == threshold up to ~1e-6 relative)."""
import numpy as np
import pytest
import torch

from oracle import hashrng
from oracle.warp import occu_bidirection_margin, occu_mask_bidirection_np

pytestmark = pytest.mark.gpu


def _flows(B, H, W, amp, seed, integer=False, sliced=False):
    f = hashrng.symmetric((B, 4, H, W), seed, amp)
    if integer:
        f = np.round(f).astype(np.float32)
    if sliced:  # the loss passes channel slices of the [B,4,h,w] flow (flow_loss.py:101-107)
        return f[:, :2], f[:, 2:], f
    return np.ascontiguousarray(f[:, :2]), np.ascontiguousarray(f[:, 2:]), None


@pytest.mark.parametrize("B,H,W,amp,integer,sliced", [
    (2, 37, 53, 0.8, False, False),   # small flows: mostly visible
    (2, 37, 53, 6.0, False, True),    # mixed, channel-slice inputs
    (1, 20, 30, 40.0, False, False),  # most samples leave the image (zeros padding)
    (2, 16, 24, 3.0, True, True),     # integer flows: taps on exact pixels
    (1, 1, 7, 2.0, False, False),     # one row (H - 1 = 0 in the normaliser)
])
def test_occ_bidirection_matches_oracle(hip_device, B, H, W, amp, integer, sliced):
    from unsamflow_amd import ops
    from unsamflow_amd.warp_utils import get_occu_mask_bidirection

    f12, f21, full = _flows(B, H, W, amp, 71, integer, sliced)
    if sliced:
        t = torch.from_numpy(full).to(hip_device)
        t12, t21 = t[:, :2], t[:, 2:]
    else:
        t12, t21 = torch.from_numpy(f12).to(hip_device), torch.from_numpy(f21).to(hip_device)
    got = get_occu_mask_bidirection(t12, t21).cpu().numpy()
    want = occu_mask_bidirection_np(f12, f21)
    near = occu_bidirection_margin(f12, f21) < 1e-5 * (1 + amp) ** 2
    assert got.shape == (B, 1, H, W)
    assert np.array_equal(got[~near], want[~near])
    # the reference's own composition on the same device: HIP zeros warp + torch test
    w = ops.warp_forward(t21.contiguous(), t12.contiguous(), "zeros")
    d = t12 + w
    mag = (t12 * t12).sum(1, keepdim=True) + (w * w).sum(1, keepdim=True)
    comp = ((d * d).sum(1, keepdim=True) > 0.01 * mag + 0.5).float()
    assert torch.equal(ops.occ_bidirection(t12, t21), comp)


def test_occ_bidirection_full_resolution(hip_device):
    """KITTI loss resolution (8 x 256 x 832), smooth +-10 px flows in opposite
    directions with a disoccluding band: against the oracle."""
    from unsamflow_amd import ops

    B, H, W = 8, 256, 832
    yy = np.linspace(0, 6.2832, H, dtype=np.float32)[None, None, :, None]
    xx = np.linspace(0, 6.2832, W, dtype=np.float32)[None, None, None, :]
    f12 = np.concatenate([10 * np.sin(xx + yy) + np.zeros((B, 1, H, W), np.float32),
                          4 * np.cos(2 * yy) + np.zeros((B, 1, H, W), np.float32)], 1).astype(np.float32)
    f21 = (-f12 + hashrng.symmetric((B, 2, H, W), 72, 1.5)).astype(np.float32)
    got = ops.occ_bidirection(torch.from_numpy(f12).to(hip_device), torch.from_numpy(f21).to(hip_device))
    want = occu_mask_bidirection_np(f12, f21)
    near = occu_bidirection_margin(f12, f21) < 1e-3
    g = got.cpu().numpy()
    assert np.array_equal(g[~near], want[~near])
    assert 0.01 < want.mean() < 0.99
