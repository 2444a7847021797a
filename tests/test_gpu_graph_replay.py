"""Hot-path calls captured into a HIP graph and replayed must give the eager
result on every replay: the library's per-call state (the binned warp
backward's zeroed counts and overflow list, the channel-split forward's
partials and sign-mask words, the photometric partials) is rebuilt by the
captured launches themselves, not by host code that a replay skips.

Decoder / loss shapes at the bench's batch (16 / 8); flows of +-2 px and a
large shift (many overflow entries in the warp backward). Tolerance: grad_x
atol 1e-5 (its overflow entries are summed with atomics), everything else
bit-identical.
"""
import pytest
import torch

from unsamflow_amd import ops
from unsamflow_amd.kernel_timer import site_launcher

pytestmark = pytest.mark.gpu


def _replayed(fn, reps=4):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fn()
    results = []
    for _ in range(reps):
        graph.replay()
        torch.cuda.synchronize()
        results.append([None if t is None else t.clone() for t in out])
    del graph
    return results


@pytest.mark.parametrize("shift", [0.0, 26.0])
@pytest.mark.parametrize("C,H,W", [(32, 64, 208), (128, 8, 26)])
def test_warp_backward_graph_replay(hip_device, C, H, W, shift):
    g = torch.Generator(device=hip_device).manual_seed(3)
    B = 16
    x = torch.randn(B, C, H, W, device=hip_device, generator=g)
    yy = torch.linspace(0, 6.2832, H, device=hip_device).view(1, 1, H, 1)
    xx = torch.linspace(0, 6.2832, W, device=hip_device).view(1, 1, 1, W)
    flow = (torch.sin(2 * xx) + torch.cos(3 * yy)).expand(B, 2, H, W).contiguous()
    flow[:, 0] += shift  # a large shift piles sources on the border column: overflow entries
    go = torch.randn(B, C, H, W, device=hip_device, generator=g)
    fn = lambda: ops.warp_backward(x, flow, go, "border", True, True)  # noqa: E731
    gx_ref, gf_ref = fn()
    torch.cuda.synchronize()
    for gx, gf in _replayed(fn):
        torch.testing.assert_close(gx, gx_ref, atol=1e-5, rtol=0)
        assert torch.equal(gf, gf_ref)


@pytest.mark.parametrize("C,H,W", [(192, 4, 13), (32, 64, 208)])
def test_corr_leaky_site_graph_replay(hip_device, C, H, W):
    # the decoder's site: forward with the sign mask (split at L0), then the backward
    def fn_factory():
        g = torch.Generator(device=hip_device).manual_seed(4)
        B = 16
        x1 = torch.randn(B, C, H, W, device=hip_device, generator=g)
        x2 = torch.randn(B, C, H, W, device=hip_device, generator=g)
        cat = torch.randn(B, 81 + C + 2, H, W, device=hip_device, generator=g)
        act = torch.empty(B, 81 + C + 2, H, W, device=hip_device)
        mask = ops.corr_act_mask(B, H, W, 4, hip_device, C=C)

        def fn():
            ops.corr_forward_ex(x1, x2, 4, act[:, :81], 0.1, act_mask=mask)
            g1, g2 = ops.corr_backward_ex(x1, x2, cat[:, :81], 4, True, True, act_out=act[:, :81], act_mask=mask)
            return act[:, :81].clone(), g1, g2
        return fn

    fn = fn_factory()
    ref = [t.clone() for t in fn()]
    torch.cuda.synchronize()
    for res in _replayed(fn):
        for a, b in zip(res, ref):
            assert torch.equal(a, b)


def test_photometric_pair_graph_replay(hip_device):
    fn = site_launcher("photo_pair_grad", (8, 3, 256, 832, "border"), hip_device)
    ref = [t.clone() for t in fn()]
    torch.cuda.synchronize()
    for res in _replayed(fn):
        for a, b in zip(res, ref):
            assert torch.equal(a, b)
