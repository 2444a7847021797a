"""Fused correlation epilogue (unsamflow_amd.corr_cat) vs the
decoder's composition cat([leaky_relu(corr(a, b)) ...] + extras) on the same
HIP correlation: forward bit-identical (same kernel arithmetic, epilogue
v > 0 ? v : 0.1 v), gradients of every input within 1e-6."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import hashrng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,H,W,n_pairs", [(2, 32, 20, 28, 1), (2, 16, 9, 26, 1), (2, 32, 16, 24, 2), (1, 8, 4, 13, 1)])
def test_corr_leaky_cat_matches_composition(hip_device, B, C, H, W, n_pairs):
    from unsamflow_amd import ops
    from unsamflow_amd.corr_cat import corr_leaky_cat

    def mk(shape, seed):
        return torch.from_numpy(hashrng.normal(shape, seed)).to(hip_device).requires_grad_(True)

    pairs = [(mk((B, C, H, W), 10 * i + 1), mk((B, C, H, W), 10 * i + 2)) for i in range(n_pairs)]
    extras = [mk((B, 32, H, W), 91), mk((B, 2, H, W), 92)]
    g = torch.from_numpy(hashrng.normal((B, 81 * n_pairs + 34, H, W), 93)).to(hip_device)

    out = corr_leaky_cat(pairs, extras, 4, 0.1)
    out.backward(g)
    got = [t.grad.clone() for p in pairs for t in p] + [e.grad.clone() for e in extras]
    for t in [t for p in pairs for t in p] + extras:
        t.grad = None

    class CorrF(torch.autograd.Function):
        @staticmethod
        def forward(ctx, a, b):
            ctx.save_for_backward(a, b)
            return ops.corr_forward(a, b, 4)

        @staticmethod
        def backward(ctx, go):
            a, b = ctx.saved_tensors
            return ops.corr_backward(a, b, go, 4)

    ref = torch.cat([F.leaky_relu(CorrF.apply(a, b), 0.1) for a, b in pairs] + extras, dim=1)
    ref.backward(g)
    want = [t.grad for p in pairs for t in p] + [e.grad for e in extras]
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref.detach().cpu().numpy())
    for a, b in zip(got, want):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("B,C,H,W", [(2, 32, 64, 208), (2, 64, 32, 104), (8, 96, 16, 52), (1, 8, 5, 4), (3, 16, 7, 12),
                                     (16, 192, 4, 13), (16, 128, 8, 26), (2, 8, 3, 5), (1, 4, 9, 1)])
def test_sign_mask_derivative_equals_dense_pass(hip_device, B, C, H, W):
    """The forward's LeakyReLU sign mask (epilogue, or the atomic OR of the
    channel-split reduce at (8, 96, 16, 52) and the KITTI L0/L1 shapes; widths
    that are not a multiple of 4 included) equals (activated output > 0) bit
    for bit, and the backward that applies the derivative from it inside its
    gradient loads gives the same gradients, bit for bit, as the dense
    derivative pass over the activated output."""
    from unsamflow_amd import ops

    x1 = torch.from_numpy(hashrng.normal((B, C, H, W), 301)).to(hip_device)
    x2 = torch.from_numpy(hashrng.normal((B, C, H, W), 302)).to(hip_device)
    buf = torch.zeros((B, 81 + 34, H, W), device=hip_device)
    out = buf[:, :81]
    mask = ops.corr_act_mask(B, H, W, 4, hip_device)
    W4 = (W + 3) // 4
    assert mask is not None and tuple(mask.shape) == (B, 9, H, W4)
    ops.corr_forward_ex(x1, x2, 4, out, 0.1, act_mask=mask)
    # expected words from the activated output: bit 4 dx + x % 4 of word (b, dy, y, x // 4)
    padded = torch.nn.functional.pad((out > 0).to(torch.int64), (0, 4 * W4 - W))
    pos = padded.view(B, 9, 9, H, W4, 4)  # b, dy, dx, y, quad, i
    shifts = (4 * torch.arange(9, device=hip_device).view(1, 1, 9, 1, 1, 1)
              + torch.arange(4, device=hip_device).view(1, 1, 1, 1, 1, 4))
    want = (pos << shifts).sum(dim=(2, 5))
    assert torch.equal(mask, want)
    g = torch.from_numpy(hashrng.normal((B, 81 + 34, H, W), 303)).to(hip_device)[:, :81]
    a1, a2 = ops.corr_backward_ex(x1, x2, g, 4, act_out=out, leaky_slope=0.1)
    m1, m2 = ops.corr_backward_ex(x1, x2, g, 4, act_out=out, leaky_slope=0.1, act_mask=mask)
    assert torch.equal(a1, m1) and torch.equal(a2, m2)
    n1, _ = ops.corr_backward_ex(x1, x2, g, 4, need_x2=False, act_mask=mask, leaky_slope=0.1)
    _, n2 = ops.corr_backward_ex(x1, x2, g, 4, need_x1=False, act_mask=mask, leaky_slope=0.1)
    assert torch.equal(n1, a1) and torch.equal(n2, a2)


@pytest.mark.parametrize("B,C,H,W", [(16, 32, 64, 208), (16, 32, 112, 256), (16, 64, 32, 104), (16, 96, 16, 52),
                                     (16, 128, 8, 26), (16, 192, 4, 13)])
def test_production_backward_site_vs_oracle(hip_device, B, C, H, W):
    """The decoder's backward call exactly as the step makes it (corr_cat:
    usf_corr_bwd_ex_f32 with the forward's sign mask, both gradients in one
    launch, gradient read from the concat gradient's slice) at the batch-16
    L4 shapes -- KITTI 64x208 and Sintel 112x256 -- and KITTI L3-L0 (L2-L0:
    the four-image ring), against the fp64 oracle (correlation_native.py:13-23
    autograd, restated in oracle.corr) with the LeakyReLU derivative taken from
    the activated output as the in-place module does (pwclite.py:307-308).
    Tolerance: atol = rtol = 1e-5 (the corr contract)."""
    from oracle.corr import corr_backward_torch64
    from unsamflow_amd import ops

    x1 = torch.from_numpy(hashrng.normal((B, C, H, W), 401)).to(hip_device)
    x2 = torch.from_numpy(hashrng.normal((B, C, H, W), 402)).to(hip_device)
    buf = torch.zeros((B, 81 + C + 2, H, W), device=hip_device)
    mask = ops.corr_act_mask(B, H, W, 4, hip_device, C=C)
    assert mask is not None  # every level carries the sign mask in production
    ops.corr_forward_ex(x1, x2, 4, buf[:, :81], 0.1, act_mask=mask)
    g = torch.from_numpy(hashrng.normal((B, 81 + C + 2, H, W), 403)).to(hip_device)
    gx1, gx2 = ops.corr_backward_ex(x1, x2, g[:, :81], 4, True, True, act_out=buf[:, :81], leaky_slope=0.1,
                                    act_mask=mask)
    act = buf[:, :81].cpu()
    g_eff = torch.where(act > 0, g[:, :81].cpu(), g[:, :81].cpu() * 0.1)
    r1, r2 = corr_backward_torch64(x1.cpu(), x2.cpu(), g_eff, 4)
    torch.testing.assert_close(gx1.cpu().double(), r1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(gx2.cpu().double(), r2, atol=1e-5, rtol=1e-5)



@pytest.mark.parametrize("B,C,H,W", [(16, 32, 64, 208), (12, 32, 40, 100), (12, 16, 40, 98), (20, 32, 24, 76)])
def test_production_forward_site_vs_oracle(hip_device, B, C, H, W):
    """The decoder's forward call as the step makes it (usf_corr_fwd_ex_f32: the
    LeakyReLU epilogue into a concat slice plus the sign mask) on grids where the
    edge-last block order of corr_fwd_kernel is active (>= USF_FWD_EDGE_MIN = 512
    workgroups and W % 32 != 0): KITTI L4 at batch 16 (896 workgroups, the
    production site) and three ragged grids of 540-720 workgroups on the other
    tile configuration, 16-byte and dword staging. Every activated value against
    the fp64 oracle (correlation_native.py:13-23, leaky_relu as pwclite.py:308),
    atol = rtol = 1e-5; every mask bit equals (activated output > 0), and equals
    the oracle's sign wherever |oracle| > 1e-5."""
    from oracle.corr import corr_forward_torch64
    from unsamflow_amd import _lib, ops

    lib = _lib.load()
    assert lib.usf_set_variant(0, -1) > 0  # the shape heuristic, not a forced candidate
    x1 = torch.from_numpy(hashrng.normal((B, C, H, W), 501)).to(hip_device)
    x2 = torch.from_numpy(hashrng.normal((B, C, H, W), 502)).to(hip_device)
    buf = torch.full((B, 81 + C + 2, H, W), float("nan"), device=hip_device)
    mask = ops.corr_act_mask(B, H, W, 4, hip_device, C=C)
    ops.corr_forward_ex(x1, x2, 4, buf[:, :81], 0.1, act_mask=mask)
    torch.cuda.synchronize()
    got = buf[:, :81].cpu()
    assert torch.isnan(buf[:, 81:]).all().item(), "forward wrote outside its concat slice"
    ref = corr_forward_torch64(x1.cpu(), x2.cpu(), 4)
    want = torch.where(ref > 0, ref, ref * 0.1)
    torch.testing.assert_close(got.double(), want, atol=1e-5, rtol=1e-5)
    W4 = (W + 3) // 4
    bits = torch.arange(4).view(1, 1, 1, 1, 1, 4) + 4 * torch.arange(9).view(1, 1, 9, 1, 1, 1)
    words = mask.cpu().view(B, 9, 1, H, W4, 1)
    mbit = ((words >> bits) & 1).bool().reshape(B, 9, 9, H, 4 * W4)[..., :W]
    mbit = mbit.reshape(B, 81, H, W)
    assert torch.equal(mbit, got > 0)
    clear = ref.abs() > 1e-5
    assert torch.equal(mbit[clear], (ref > 0)[clear])


@pytest.mark.parametrize("masked", [False, True])
def test_backward_ring_dword_steady_state_vs_oracle(hip_device, masked):
    """The four-image ring's steady-state wait (bwd_wait_stages<F, NB-2, 0>, reached
    only with >= 4 stages per workgroup) on the dword-DMA path, whose per-wave
    chunk counts differ by wave (advisor r04): (16, 192, 16, 50) is 128 units
    (ring), 4 channel groups of 48 channels = 12 stages, W % 4 = 2 (dword DMA).
    Plain backward and the decoder's masked form, against the fp64 oracle
    (correlation_cuda_kernel.cu:116-300 via oracle.corr), atol = rtol = 1e-5."""
    from oracle.corr import corr_backward_torch64
    from unsamflow_amd import ops

    B, C, H, W = 16, 192, 16, 50
    x1 = torch.from_numpy(hashrng.normal((B, C, H, W), 601)).to(hip_device)
    x2 = torch.from_numpy(hashrng.normal((B, C, H, W), 602)).to(hip_device)
    g = torch.from_numpy(hashrng.normal((B, 81, H, W), 603)).to(hip_device)
    if masked:
        buf = torch.zeros((B, 81, H, W), device=hip_device)
        mask = ops.corr_act_mask(B, H, W, 4, hip_device, C=C)
        ops.corr_forward_ex(x1, x2, 4, buf, 0.1, act_mask=mask)
        gx1, gx2 = ops.corr_backward_ex(x1, x2, g, 4, True, True, leaky_slope=0.1, act_mask=mask)
        act = buf.cpu()
        g_ref = torch.where(act > 0, g.cpu(), g.cpu() * 0.1)
    else:
        gx1, gx2 = ops.corr_backward(x1, x2, g, 4)
        g_ref = g.cpu()
    r1, r2 = corr_backward_torch64(x1.cpu(), x2.cpu(), g_ref, 4)
    torch.testing.assert_close(gx1.cpu().double(), r1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(gx2.cpu().double(), r2, atol=1e-5, rtol=1e-5)
