"""Decoder flow upsampling (unsamflow_amd.upsample) vs the
reference operator itself -- torch's F.interpolate(flow * k, scale_factor=k,
mode="bilinear", align_corners=True) on the CPU -- forward and backward."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import hashrng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,k", [((16, 2, 4, 13), 2), ((16, 2, 32, 104), 2), ((16, 2, 64, 208), 4),
                                     ((2, 2, 1, 5), 2), ((3, 3, 7, 9), 4), ((1, 2, 5, 1), 2)])
def test_flow_upsample_matches_torch(hip_device, shape, k):
    from unsamflow_amd.upsample import upsample_flow

    f = torch.from_numpy(hashrng.symmetric(shape, 77 + shape[2], 20.0))
    go = torch.from_numpy(hashrng.normal((shape[0], shape[1], shape[2] * k, shape[3] * k), 78))
    fr = f.clone().requires_grad_(True)
    ref = F.interpolate(fr * k, scale_factor=k, mode="bilinear", align_corners=True)
    ref.backward(go)
    fd = f.to(hip_device).requires_grad_(True)
    out = upsample_flow(fd, k)
    out.backward(go.to(hip_device))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=2e-5, rtol=1e-6)
    np.testing.assert_allclose(fd.grad.cpu().numpy(), fr.grad.numpy(), atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("B,C,H,W", [(2, 3, 256, 832), (1, 3, 448, 1024), (3, 1, 8, 16), (2, 3, 24, 40)])
def test_area_pyramid_bit_exact_vs_torch_cpu(hip_device, B, C, H, W):
    """usf_area_pyramid_f32 == F.interpolate(x, (H >> s, W >> s), mode="area")
    on the CPU (torch's row-major block sum, / k / k), bit for bit."""
    import torch.nn.functional as F

    from oracle import hashrng
    from unsamflow_amd import ops

    x = torch.from_numpy(hashrng.uniform((B, C, H, W), 77 + H))
    outs = ops.area_pyramid(x.to(hip_device))
    for s, o in zip((1, 2, 3), outs):
        ref = F.interpolate(x, (H >> s, W >> s), mode="area")
        assert torch.equal(o.cpu(), ref), (s, float((o.cpu() - ref).abs().max()))


@pytest.mark.parametrize("B,H,W,f", [(2, 5, 7, 4), (1, 1, 1, 4), (8, 4, 13, 4), (2, 64, 208, 4), (3, 9, 70, 4),
                                     (1, 6, 9, 2), (1, 3, 5, 8)])
def test_convex_upsample_matches_oracle(hip_device, B, H, W, f):
    """usf_convex_upsample_{f32,bwd_f32} vs oracle/upsample.py (UpFlowNetwork,
    pwclite.py:140-166): fp32 kernel vs fp64 oracle, atol 1e-4 + rtol 1e-5 on
    outputs of magnitude ~100."""
    from oracle.upsample import convex_upsample_backward_np, convex_upsample_np
    from unsamflow_amd.upsample import convex_upsample

    flow = hashrng.symmetric((B, 2, H, W), 400 + H, 20.0)
    mask = hashrng.normal((B, 9 * f * f, H, W), 401 + W) * np.float32(3.0)
    gout = hashrng.normal((B, 2, f * H, f * W), 402)
    fd = torch.from_numpy(flow).to(hip_device).requires_grad_(True)
    md = torch.from_numpy(mask).to(hip_device).requires_grad_(True)
    out = convex_upsample(fd, md, f, 0.25)
    out.backward(torch.from_numpy(gout).to(hip_device))
    np.testing.assert_allclose(out.detach().cpu().numpy(), convex_upsample_np(flow, mask, f, 0.25),
                               atol=1e-4, rtol=1e-5)
    gf, gm = convex_upsample_backward_np(flow, mask, gout, f, 0.25)
    np.testing.assert_allclose(fd.grad.cpu().numpy(), gf, atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(md.grad.cpu().numpy(), gm, atol=1e-4, rtol=1e-5)


def test_convex_upsample_deterministic_and_partial_grads(hip_device):
    from unsamflow_amd import ops

    B, H, W, f = 2, 64, 208, 4
    flow = torch.from_numpy(hashrng.symmetric((B, 2, H, W), 410, 20.0)).to(hip_device)
    mask = torch.from_numpy(hashrng.normal((B, 144, H, W), 411)).to(hip_device)
    go = torch.from_numpy(hashrng.normal((B, 2, f * H, f * W), 412)).to(hip_device)
    a = ops.convex_upsample_backward(flow, mask, go, f)
    b = ops.convex_upsample_backward(flow, mask, go, f)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    gf, gm = ops.convex_upsample_backward(flow, mask, go, f, need_mask=False)
    assert gm is None and torch.equal(gf, a[0])
    gf, gm = ops.convex_upsample_backward(flow, mask, go, f, need_flow=False)
    assert gf is None and torch.equal(gm, a[1])


def test_upflow_network_fused_matches_torch_form(hip_device):
    """The model's UpFlowNetwork with the HIP op vs its torch form (pwclite.py:
    148-166) on the device, including the convs' parameter gradients."""
    from unsamflow_amd.pwclite import UpFlowNetwork

    torch.manual_seed(0)
    net = UpFlowNetwork(96, 4).to(hip_device)
    flow = torch.randn(2, 2, 16, 52, device=hip_device) * 5
    feat = torch.randn(2, 96, 16, 52, device=hip_device)
    go = torch.randn(2, 2, 64, 208, device=hip_device)
    outs, grads = [], []
    for fused in (False, True):
        net.fused = fused
        net.zero_grad()
        fl = flow.clone().requires_grad_(True)
        out = net(fl, feat)
        out.backward(go)
        outs.append(out.detach())
        grads.append([fl.grad] + [p.grad.clone() for p in net.parameters()])
    torch.testing.assert_close(outs[1], outs[0], atol=1e-4, rtol=1e-5)
    for a, b in zip(grads[1], grads[0]):
        torch.testing.assert_close(a, b, atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("B,sizes", [(16, [(64, 208), (32, 104), (16, 52), (8, 26), (4, 13)]),
                                     (3, [(9, 7), (5, 4), (1, 1)])])
def test_convex_pyramid_equals_per_level_calls(hip_device, B, sizes):
    """convex_upsample_pyramid (usf_convex_upsample_pyramid_{f32,bwd_f32}:
    every decoder level in one launch each way) gives the per-level
    convex_upsample results bit for bit -- outputs, grad_flow and grad_mask --
    at the decoder's batch-16 KITTI levels and odd sizes (incl. 1x1)."""
    from unsamflow_amd.upsample import convex_upsample, convex_upsample_pyramid

    gen = torch.Generator(device=hip_device).manual_seed(11)
    flows = [torch.randn(B, 2, h, w, device=hip_device, generator=gen) for h, w in sizes]
    masks = [torch.randn(B, 144, h, w, device=hip_device, generator=gen) for h, w in sizes]
    gos = [torch.randn(B, 2, 4 * h, 4 * w, device=hip_device, generator=gen) for h, w in sizes]
    fa = [f.clone().requires_grad_(True) for f in flows]
    ma = [m.clone().requires_grad_(True) for m in masks]
    fb = [f.clone().requires_grad_(True) for f in flows]
    mb = [m.clone().requires_grad_(True) for m in masks]
    ups = convex_upsample_pyramid(fa, ma, 4, 0.25)
    refs = [convex_upsample(f, m, 4, 0.25) for f, m in zip(fb, mb)]
    for u, r in zip(ups, refs):
        assert torch.equal(u, r)
    sum((u * g).sum() for u, g in zip(ups, gos)).backward()
    sum((r * g).sum() for r, g in zip(refs, gos)).backward()
    for a, b in zip(fa + ma, fb + mb):
        assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("pad", ["border", "zeros"])
@pytest.mark.parametrize("B,C,H,W", [(16, 128, 8, 26), (16, 32, 64, 208), (3, 5, 14, 32)])
def test_upsample_warp_equals_separate_calls(hip_device, B, C, H, W, pad):
    """usf_warp_fwd_up_f32 (the decoder's x2 upsampling + flow_warp of x2 in one
    launch, pwclite.py:299-302) gives the same numbers as usf_flow_upsample_f32
    followed by usf_warp_fwd_f32, bit for bit; its autograd form gives the
    gradients of the two-op form (to the rounding of the binned gather's
    overflow atomics and of the gradient sum order)."""
    from unsamflow_amd import ops
    from unsamflow_amd.upsample import upsample_flow, upsample_warp
    from unsamflow_amd.warp_utils import flow_warp

    coarse = torch.from_numpy(hashrng.symmetric((B, 2, H // 2, W // 2), 430 + C, 3.0)).to(hip_device)
    x = torch.from_numpy(hashrng.normal((B, C, H, W), 431 + C)).to(hip_device)
    g_up = torch.from_numpy(hashrng.normal((B, 2, H, W), 432 + C)).to(hip_device)
    g_out = torch.from_numpy(hashrng.normal((B, C, H, W), 433 + C)).to(hip_device)
    up_ref = ops.flow_upsample(coarse, 2)
    out_ref = ops.warp_forward(x, up_ref, pad)
    up, out = ops.warp_forward_up(x, coarse, pad)
    assert torch.equal(up, up_ref) and torch.equal(out, out_ref)

    c1, x1 = coarse.clone().requires_grad_(True), x.clone().requires_grad_(True)
    u1 = upsample_flow(c1, 2)
    o1 = flow_warp(x1, u1, pad)
    torch.autograd.backward([u1, o1], [g_up, g_out])
    c2, x2 = coarse.clone().requires_grad_(True), x.clone().requires_grad_(True)
    u2, o2 = upsample_warp(c2, x2, pad)
    assert torch.equal(u2, u1) and torch.equal(o2, o1)
    torch.autograd.backward([u2, o2], [g_up, g_out])
    # grad_x: cells with more than 4 sources (this random +-6 px field has them)
    # add their excess with fp32 atomics, so two calls agree to rounding only
    torch.testing.assert_close(x2.grad, x1.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(c2.grad, c1.grad, atol=1e-5, rtol=1e-6)


@pytest.mark.parametrize("shape", [(16, 2, 8, 26), (16, 2, 64, 208), (3, 2, 5, 7)])
def test_upsample_backward_of_a_sum_is_bit_exact(hip_device, shape):
    """usf_flow_upsample_bwd_sum_f32(a, b) == usf_flow_upsample_bwd_f32(a + b):
    the per-element add inside the gather is the same IEEE add."""
    from unsamflow_amd import ops

    B, C, h, w = shape
    a = torch.from_numpy(hashrng.normal((B, C, 2 * h, 2 * w), 440)).to(hip_device)
    b = torch.from_numpy(hashrng.normal((B, C, 2 * h, 2 * w), 441)).to(hip_device)
    assert torch.equal(ops.flow_upsample_backward(a, 2, b), ops.flow_upsample_backward(a + b, 2))
