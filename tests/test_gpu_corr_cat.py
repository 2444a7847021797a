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
