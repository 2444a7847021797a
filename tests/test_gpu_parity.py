"""Parity of the HIP kernels (through the C ABI) with the oracle and the
reference's golden vectors. Runs on an MI355X: ``pytest -m gpu``.

Tolerances (fp32; stated per SURVEY.md §8c):
* correlation fwd/bwd: atol=1e-5, rtol=1e-5 vs the reference / fp64 oracle;
* warp fwd: atol=1e-5; warp grad_flow: atol=1e-4, rtol=1e-5; warp grad_x:
  atol=1e-4, rtol=1e-5 (fp32 atomics: the order in which the up-to-dozens of
  source pixels add into one grad_x element is not fixed).
"""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle import hashrng
from oracle.corr import corr_backward_np, corr_forward_np
from oracle.warp import warp_backward_np, warp_forward_np

pytestmark = pytest.mark.gpu

CORR_ATOL = 1e-5
CORR_RTOL = 1e-5


def _dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    return t.detach().cpu().numpy()


# ------------------------------------------------------------ correlation --
@pytest.mark.parametrize("name", golden_files("corr_"))
def test_corr_fwd_bwd_vs_reference_golden(hip_device, name):
    from unsamflow_amd import ops

    z = load_golden(name)
    d = int(z["d"])
    x1, x2, g = _dev(z["x1"], hip_device), _dev(z["x2"], hip_device), _dev(z["gout"], hip_device)
    out = ops.corr_forward(x1, x2, d)
    gx1, gx2 = ops.corr_backward(x1, x2, g, d)
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(out), z["out"], atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(gx1), z["gx1"], atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(gx2), z["gx2"], atol=CORR_ATOL, rtol=CORR_RTOL)


# shapes of every PWCLite call site (KITTI + Sintel levels, mask-feature C=32),
# plus ragged edges; B kept small so the fp64 oracle stays fast
FUZZ_SHAPES = [
    (2, 192, 4, 13), (2, 128, 8, 26), (1, 96, 16, 52), (1, 64, 32, 104), (1, 32, 64, 208),
    (1, 192, 7, 16), (1, 128, 14, 32), (1, 32, 28, 64), (1, 32, 4, 13),
    (3, 5, 17, 33), (1, 1, 1, 1), (1, 17, 2, 70), (2, 40, 9, 9), (1, 8, 65, 3),
]


@pytest.mark.parametrize("shape", FUZZ_SHAPES)
def test_corr_vs_oracle_call_site_shapes(hip_device, shape):
    from unsamflow_amd import ops

    B, C, H, W = shape
    seed = B * 1000003 + C * 1009 + H * 31 + W
    x1 = hashrng.normal(shape, seed)
    x2 = hashrng.normal(shape, seed + 1)
    g = hashrng.normal((B, 81, H, W), seed + 2)
    t1, t2, tg = _dev(x1, hip_device), _dev(x2, hip_device), _dev(g, hip_device)
    out = ops.corr_forward(t1, t2, 4)
    gx1, gx2 = ops.corr_backward(t1, t2, tg, 4)
    np.testing.assert_allclose(_np(out), corr_forward_np(x1, x2, 4), atol=CORR_ATOL, rtol=CORR_RTOL)
    r1, r2 = corr_backward_np(x1, x2, g, 4)
    np.testing.assert_allclose(_np(gx1), r1, atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(gx2), r2, atol=CORR_ATOL, rtol=CORR_RTOL)


@pytest.mark.parametrize("d", [1, 2, 3])
def test_corr_other_displacements_vs_oracle(hip_device, d):
    from unsamflow_amd import ops

    shape = (2, 24, 19, 45)
    x1 = hashrng.normal(shape, 11 + d)
    x2 = hashrng.normal(shape, 22 + d)
    K = 2 * d + 1
    g = hashrng.normal((2, K * K, 19, 45), 33 + d)
    t1, t2 = _dev(x1, hip_device), _dev(x2, hip_device)
    out = ops.corr_forward(t1, t2, d)
    gx1, gx2 = ops.corr_backward(t1, t2, _dev(g, hip_device), d)
    np.testing.assert_allclose(_np(out), corr_forward_np(x1, x2, d), atol=CORR_ATOL, rtol=CORR_RTOL)
    r1, r2 = corr_backward_np(x1, x2, g, d)
    np.testing.assert_allclose(_np(gx1), r1, atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(gx2), r2, atol=CORR_ATOL, rtol=CORR_RTOL)


@pytest.mark.parametrize("name", golden_files("corrbig_"))
def test_corr_full_size_configs_vs_reference(hip_device, name):
    """BASELINE configs 1 and 2 at full size: reference sums + 4096 sampled elements."""
    from unsamflow_amd import ops

    z = load_golden(name)
    B, C, H, W, d, seed = (int(v) for v in z["shape"])
    x1 = _dev(hashrng.normal((B, C, H, W), seed), hip_device)
    x2 = _dev(hashrng.normal((B, C, H, W), seed + 1), hip_device)
    g = _dev(hashrng.normal((B, (2 * d + 1) ** 2, H, W), seed + 2), hip_device)
    out = ops.corr_forward(x1, x2, d)
    gx1, gx2 = ops.corr_backward(x1, x2, g, d)
    for key, t in (("out", out), ("gx1", gx1), ("gx2", gx2)):
        flat = t.reshape(-1)
        idx = torch.from_numpy(z[key + "_idx"]).to(hip_device)
        np.testing.assert_allclose(_np(flat[idx]), z[key + "_val"], atol=CORR_ATOL, rtol=CORR_RTOL)
        s = flat.double().sum().item()
        a = flat.double().abs().sum().item()
        assert abs(s - float(z[key + "_sum"])) <= 1e-5 * float(z[key + "_abssum"]), key
        assert abs(a - float(z[key + "_abssum"])) <= 1e-5 * float(z[key + "_abssum"]), key


def test_corr_backward_is_deterministic(hip_device):
    from unsamflow_amd import ops

    shape = (2, 64, 32, 104)
    x1 = _dev(hashrng.normal(shape, 5), hip_device)
    x2 = _dev(hashrng.normal(shape, 6), hip_device)
    g = _dev(hashrng.normal((2, 81, 32, 104), 7), hip_device)
    a1, a2 = ops.corr_backward(x1, x2, g, 4)
    b1, b2 = ops.corr_backward(x1, x2, g, 4)
    assert torch.equal(a1, b1) and torch.equal(a2, b2)


def test_corr_properties_at_kitti_l4_full_batch(hip_device):
    """Size-independent properties at the largest call site (B=8, C=32, 64x208):
    bilinearity of the forward, the adjoint identity <corr(x1,x2), g> =
    <x1, gx1> = <x2, gx2>, and the zero-displacement channel == channel mean."""
    from unsamflow_amd import ops

    shape = (8, 32, 64, 208)
    x1 = _dev(hashrng.normal(shape, 91), hip_device)
    x2 = _dev(hashrng.normal(shape, 92), hip_device)
    x3 = _dev(hashrng.normal(shape, 93), hip_device)
    g = _dev(hashrng.normal((8, 81, 64, 208), 94), hip_device)
    o12 = ops.corr_forward(x1, x2, 4)
    o13 = ops.corr_forward(x1, x3, 4)
    o1s = ops.corr_forward(x1, 2.0 * x2 - 0.5 * x3, 4)
    torch.testing.assert_close(o1s, 2.0 * o12 - 0.5 * o13, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(o12[:, 40], (x1 * x2).mean(1), atol=1e-6, rtol=1e-5)
    gx1, gx2 = ops.corr_backward(x1, x2, g, 4)
    lhs = (o12.double() * g.double()).sum()
    r1 = (x1.double() * gx1.double()).sum()
    r2 = (x2.double() * gx2.double()).sum()
    scale = (o12.double().abs() * g.double().abs()).sum()
    assert abs(lhs - r1) <= 1e-6 * scale
    assert abs(lhs - r2) <= 1e-6 * scale


def test_correlation_module_autograd_and_inplace_relu(hip_device):
    """Module path as PWCLite uses it: in-place LeakyReLU on the output, then backward."""
    from unsamflow_amd.correlation import Correlation

    shape = (2, 16, 12, 20)
    x1 = hashrng.normal(shape, 71)
    x2 = hashrng.normal(shape, 72)
    g = hashrng.normal((2, 81, 12, 20), 73)
    t1 = _dev(x1, hip_device).requires_grad_(True)
    t2 = _dev(x2, hip_device).requires_grad_(True)
    corr = Correlation(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=1)
    out = torch.nn.LeakyReLU(0.1, inplace=True)(corr(t1, t2))
    out.backward(_dev(g, hip_device))
    ref = corr_forward_np(x1, x2, 4)
    np.testing.assert_allclose(_np(out), np.where(ref > 0, ref, 0.1 * ref), atol=CORR_ATOL, rtol=CORR_RTOL)
    gr = np.where(ref > 0, g, 0.1 * g)
    r1, r2 = corr_backward_np(x1, x2, gr, 4)
    np.testing.assert_allclose(_np(t1.grad), r1, atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(t2.grad), r2, atol=CORR_ATOL, rtol=CORR_RTOL)


def test_correlation_only_one_input_requires_grad(hip_device):
    from unsamflow_amd.correlation_native import Correlation

    t1 = _dev(hashrng.normal((1, 8, 6, 9), 1), hip_device).requires_grad_(True)
    t2 = _dev(hashrng.normal((1, 8, 6, 9), 2), hip_device)
    Correlation(4)(t1, t2).sum().backward()
    assert t1.grad is not None and t2.grad is None


def test_corr_noncontiguous_inputs(hip_device):
    from unsamflow_amd import ops

    base = _dev(hashrng.normal((2, 20, 10, 12), 3), hip_device)
    x1 = base[:, ::2]
    x2 = base[:, 1::2]
    out = ops.corr_forward(x1, x2, 4)
    ref = corr_forward_np(_np(x1), _np(x2), 4)
    np.testing.assert_allclose(_np(out), ref, atol=CORR_ATOL, rtol=CORR_RTOL)


# ------------------------------------------------------------------- warp --
def _warp_case(z, dev):
    flow_full = _dev(z["flow_full"], dev)
    flow = flow_full[:, 2:] if int(z["slice"]) else flow_full
    return _dev(z["x"], dev), flow_full, flow, str(z["pad"])


@pytest.mark.parametrize("name", golden_files("warp_"))
def test_warp_fwd_bwd_vs_reference_golden(hip_device, name):
    from unsamflow_amd.warp_utils import flow_warp

    z = load_golden(name)
    x, flow_full, flow, pad = _warp_case(z, hip_device)
    x.requires_grad_(True)
    flow_full.requires_grad_(True)
    fl = flow_full[:, 2:] if int(z["slice"]) else flow_full
    out = flow_warp(x, fl, pad=pad)
    out.backward(_dev(z["gout"], hip_device))
    gflow = _np(flow_full.grad)
    if int(z["slice"]):
        assert np.all(gflow[:, :2] == 0)
        gflow = gflow[:, 2:]
    np.testing.assert_allclose(_np(out), z["out"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(_np(x.grad), z["gx"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(gflow, z["gflow"], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("pad", ["border", "zeros"])
@pytest.mark.parametrize("shape,scale", [
    ((8, 32, 64, 208), 3.0), ((2, 3, 256, 832), 40.0), ((4, 128, 8, 26), 1.5),
    ((8, 64, 32, 104), 2.5), ((2, 5, 9, 7), 3.0), ((1, 96, 16, 52), 8.0),
])
def test_warp_vs_oracle_call_site_shapes(hip_device, pad, shape, scale):
    from unsamflow_amd import ops

    B, C, H, W = shape
    seed = C * 7 + H
    x = hashrng.uniform(shape, seed)
    flow = hashrng.symmetric((B, 2, H, W), seed + 1, scale)
    g = hashrng.normal(shape, seed + 2)
    tx, tf, tg = _dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device)
    out = ops.warp_forward(tx, tf, pad)
    gx, gf = ops.warp_backward(tx, tf, tg, pad)
    np.testing.assert_allclose(_np(out), warp_forward_np(x, flow, pad), atol=1e-5, rtol=0)
    rx, rf = warp_backward_np(x, flow, g, pad)
    np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)


def test_warp_loss_style_slices_and_flow_only_grad(hip_device):
    """flow_loss.py:130-131: image warps by channel slices of a [B,4,h,w] flow,
    gradient only w.r.t. the flow (images do not require grad)."""
    from unsamflow_amd.warp_utils import flow_warp

    B, H, W = 2, 64, 208
    im = _dev(hashrng.uniform((B, 3, H, W), 1), hip_device)
    flow4 = _dev(hashrng.symmetric((B, 4, H, W), 2, 5.0), hip_device).requires_grad_(True)
    g1 = hashrng.normal((B, 3, H, W), 3)
    g2 = hashrng.normal((B, 3, H, W), 4)
    o1 = flow_warp(im, flow4[:, :2], pad="border")
    o2 = flow_warp(im, flow4[:, 2:], pad="border")
    (o1 * _dev(g1, hip_device) + o2 * _dev(g2, hip_device)).sum().backward()
    f = _np(flow4.detach())
    imn = _np(im)
    _, r1 = warp_backward_np(imn, f[:, :2], g1, "border", need_x=False)
    _, r2 = warp_backward_np(imn, f[:, 2:], g2, "border", need_x=False)
    np.testing.assert_allclose(_np(flow4.grad), np.concatenate([r1, r2], 1), atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(_np(o1), warp_forward_np(imn, f[:, :2]), atol=1e-5, rtol=0)


def test_warp_zero_flow_is_identity(hip_device):
    from unsamflow_amd import ops

    x = _dev(hashrng.uniform((3, 16, 33, 47), 9), hip_device)
    z = torch.zeros(3, 2, 33, 47, device=hip_device)
    for pad in ("border", "zeros"):
        # the reference's normalise/unnormalise round trip moves the sample point by a few
        # ulp of the coordinate, so "identity" holds to ~|x[i+1]-x[i]| * 4 ulp
        torch.testing.assert_close(ops.warp_forward(x, z, pad), x, atol=5e-6, rtol=0)


def test_warp_integer_shift_matches_roll(hip_device):
    """An integer flow is an exact shift (bilinear weights 0/1) with border clamp."""
    from unsamflow_amd import ops

    x = _dev(hashrng.uniform((1, 4, 20, 30), 10), hip_device)
    flow = torch.zeros(1, 2, 20, 30, device=hip_device)
    flow[:, 0] = 3.0
    flow[:, 1] = -2.0
    out = ops.warp_forward(x, flow, "border")
    cols = torch.clamp(torch.arange(30, device=hip_device) + 3, 0, 29)
    rows = torch.clamp(torch.arange(20, device=hip_device) - 2, 0, 19)
    ref = x[:, :, rows][:, :, :, cols]
    torch.testing.assert_close(out, ref, atol=5e-6, rtol=0)


def test_correlation_cuda_shim_reference_call_pattern(hip_device):
    """The reference's correlation.py:9-72 call sequence against the
    correlation_cuda-compatible shim: empty tensors from .new(), resized and
    filled by the callee, return value 1."""
    from unsamflow_amd import correlation_cuda

    shape = (2, 16, 9, 30)
    x1 = hashrng.normal(shape, 41)
    x2 = hashrng.normal(shape, 42)
    g = hashrng.normal((2, 81, 9, 30), 43)
    t1, t2 = _dev(x1, hip_device), _dev(x2, hip_device)
    rbot1, rbot2, output = t1.new(), t2.new(), t1.new()
    assert correlation_cuda.forward(t1, t2, rbot1, rbot2, output, 4, 1, 4, 1, 1, 1) == 1
    np.testing.assert_allclose(_np(output), corr_forward_np(x1, x2, 4), atol=CORR_ATOL, rtol=CORR_RTOL)
    gi1, gi2 = t1.new(), t2.new()
    assert correlation_cuda.backward(t1, t2, t1.new(), t2.new(), _dev(g, hip_device), gi1, gi2, 4, 1, 4, 1, 1, 1) == 1
    r1, r2 = corr_backward_np(x1, x2, g, 4)
    np.testing.assert_allclose(_np(gi1), r1, atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(gi2), r2, atol=CORR_ATOL, rtol=CORR_RTOL)
    with pytest.raises(NotImplementedError):
        correlation_cuda.forward(t1, t2, rbot1, rbot2, output, 3, 3, 20, 1, 2, 1)


@pytest.mark.parametrize("shape", [(2, 40, 13, 37), (1, 192, 4, 13), (2, 32, 64, 70), (2, 24, 24, 64)])
def test_corr_every_tile_variant_vs_oracle(hip_device, shape):
    """Every d=4 tile variant reachable through usf_set_variant computes the same result."""
    from unsamflow_amd import _lib, ops

    lib = _lib.load()
    B, C, H, W = shape
    x1 = hashrng.normal(shape, 61)
    x2 = hashrng.normal(shape, 62)
    g = hashrng.normal((B, 81, H, W), 63)
    t1, t2, tg = _dev(x1, hip_device), _dev(x2, hip_device), _dev(g, hip_device)
    ref = corr_forward_np(x1, x2, 4)
    r1, r2 = corr_backward_np(x1, x2, g, 4)
    try:
        for v in range(lib.usf_set_variant(0, -1)):
            lib.usf_set_variant(0, v)
            np.testing.assert_allclose(_np(ops.corr_forward(t1, t2, 4)), ref, atol=CORR_ATOL, rtol=CORR_RTOL,
                                       err_msg=f"fwd variant {v}")
        for v in range(lib.usf_set_variant(1, -1)):
            lib.usf_set_variant(1, v)
            gx1, gx2 = ops.corr_backward(t1, t2, tg, 4)
            np.testing.assert_allclose(_np(gx1), r1, atol=CORR_ATOL, rtol=CORR_RTOL, err_msg=f"bwd variant {v}")
            np.testing.assert_allclose(_np(gx2), r2, atol=CORR_ATOL, rtol=CORR_RTOL, err_msg=f"bwd variant {v}")
    finally:
        lib.usf_set_variant(0, -1)
        lib.usf_set_variant(1, -1)


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_warp_grad_x_variants(hip_device, variant):
    """Every grad_x path reachable through usf_set_variant(2, .) -- the
    per-pixel lane-merged scatter, the pixel-pair scatter (the workspace-free
    entry's defaults) and the binned gather -- matches the oracle, including a
    large-flow case (many sources per cell: overflow entries)."""
    from unsamflow_amd import _lib, ops

    lib = _lib.load()
    try:
        lib.usf_set_variant(2, variant)
        for shape, scale, seed in [((2, 32, 24, 40), 2.0, 1), ((1, 64, 16, 52), 25.0, 2), ((2, 3, 33, 17), 6.0, 3),
                                   ((2, 20, 9, 70), 1.0, 4)]:
            x = hashrng.uniform(shape, 300 + seed)
            flow = hashrng.symmetric((shape[0], 2) + shape[2:], 400 + seed, scale)
            g = hashrng.normal(shape, 500 + seed)
            gx, gf = ops.warp_backward(_dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device), "border")
            rx, rf = warp_backward_np(x, flow, g, "border")
            np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
            np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)
    finally:
        lib.usf_set_variant(2, -1)


# ---------------------------------------------------------------- occlusion --
def _occ_flow_dev(z, dev):
    f = torch.from_numpy(z["flow_full"]).to(dev)
    return f[:, 2:] if int(z["slice"]) else f


def _assert_occ_equal(occ, ref, cmap_ref, th=0.2, eps=1e-5):
    """Masks equal except where the reference map sits within eps of the threshold
    (fp32 atomics sum in a different order than scatter_add_)."""
    bad = occ != ref
    assert not np.any(bad & (np.abs(np.clip(cmap_ref, 0, 1) - th) > eps)), int(bad.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_files("occ_"))
def test_occlusion_vs_reference_golden(hip_device, name):
    """usf_splat_map_f32 / usf_occ_backward_f32 vs the reference's
    get_corresponding_map / get_occu_mask_backward captures."""
    from unsamflow_amd import warp_utils

    z = load_golden(name)
    flow = _occ_flow_dev(z, hip_device)
    B, _, H, W = flow.shape
    ys, xs = torch.meshgrid(torch.arange(H, device=hip_device), torch.arange(W, device=hip_device), indexing="ij")
    coords = torch.stack([xs, ys], 0).float().expand(B, 2, H, W) + flow
    cmap = warp_utils.get_corresponding_map(coords)
    np.testing.assert_allclose(_np(cmap), z["map"], atol=2e-6, rtol=1e-6)
    occ = warp_utils.get_occu_mask_backward(flow, th=0.2)
    _assert_occ_equal(_np(occ), z["occ"], z["map"])


@pytest.mark.gpu
@pytest.mark.parametrize("shape,scale", [((8, 256, 832), 4.0), ((8, 256, 832), 0.0), ((2, 64, 208), 30.0),
                                         ((3, 33, 17), 2.5)])
def test_occlusion_vs_oracle_full_size(hip_device, shape, scale):
    """The loss's call site ([B,2,256,832] backward flow, B=8) and odd shapes vs the
    oracle; relative-displacement form vs absolute-coordinate form."""
    from oracle.torch_ref import oracle_corresponding_map, oracle_occu_mask_backward
    from unsamflow_amd import ops

    B, H, W = shape
    flow = torch.from_numpy(hashrng.symmetric((B, 2, H, W), 9100 + H, scale)) if scale else torch.zeros(B, 2, H, W)
    occ = ops.occ_backward(flow.to(hip_device), 0.2)
    ref = oracle_occu_mask_backward(flow, 0.2)
    ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    coords = torch.stack([xs, ys], 0).float().expand(B, 2, H, W) + flow
    cmap_ref = oracle_corresponding_map(coords).numpy()
    _assert_occ_equal(_np(occ), ref.numpy(), cmap_ref)
    rel = _np(ops.splat_map(flow.to(hip_device)))
    absm = _np(ops.splat_map(coords.to(hip_device), absolute=True))
    np.testing.assert_allclose(rel, cmap_ref, atol=2e-6, rtol=1e-6)
    np.testing.assert_allclose(absm, cmap_ref, atol=2e-6, rtol=1e-6)
    # mass conservation: every in-image target spreads exactly its weights
    assert abs(float(rel.sum()) - float(cmap_ref.sum())) < 1e-3 * max(1.0, float(cmap_ref.sum()))


@pytest.mark.parametrize("name", golden_files("occ_"))
def test_occ_vis_pair_vs_reference_golden(hip_device, name):
    """ops.occ_vis_pair (usf_occ_vis_pair_persist_f32: both directions' 1 -
    get_occu_mask_backward from one [B,4,H,W] flow) against the reference's
    get_occu_mask_backward captures: the captured flow as either half of the
    4-channel flow, the other half a different field (so each half must come
    from its own channels)."""
    from unsamflow_amd import ops

    z = load_golden(name)
    flow = _occ_flow_dev(z, hip_device).contiguous()
    other = torch.flip(flow, dims=[-1]).contiguous() * 0.5
    for first in (True, False):
        flow4 = torch.cat([other, flow] if first else [flow, other], 1)
        vis = ops.occ_vis_pair(flow4, 0.2)
        got = vis[0] if first else vis[1]  # vis[0] from channels 2:4, vis[1] from channels 0:2
        _assert_occ_equal(1.0 - _np(got), z["occ"], z["map"])


@pytest.mark.parametrize("shape,scale", [((8, 256, 832), 4.0), ((8, 256, 832), 0.0), ((2, 64, 208), 30.0),
                                         ((3, 33, 17), 2.5)])
def test_occ_vis_pair_vs_oracle_full_size(hip_device, shape, scale):
    """The loss's call site (both masks of a B=8 [B,4,256,832] flow) vs the oracle,
    called twice on one persistent map (the threshold pass leaves it zero)."""
    from oracle.torch_ref import oracle_corresponding_map, oracle_occu_mask_backward
    from unsamflow_amd import ops

    B, H, W = shape
    f4 = torch.from_numpy(hashrng.symmetric((B, 4, H, W), 9200 + H, scale)) if scale else torch.zeros(B, 4, H, W)
    ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    grid = torch.stack([xs, ys], 0).float().expand(B, 2, H, W)
    for _ in range(2):
        vis = ops.occ_vis_pair(f4.to(hip_device), 0.2)
        for d, half in ((0, f4[:, 2:]), (1, f4[:, :2])):
            ref = oracle_occu_mask_backward(half.contiguous(), 0.2)
            cmap_ref = oracle_corresponding_map(grid + half).numpy()
            _assert_occ_equal(1.0 - _np(vis[d]), ref.numpy(), cmap_ref)
    torch.cuda.synchronize()
    ws, _ = ops._PERSIST[(hip_device.index, "occ_vis_pair", (B, H, W))]
    assert int(torch.count_nonzero(ws)) == 0


@pytest.mark.parametrize("shape,split", [((16, 192, 4, 13), False), ((16, 128, 8, 26), False),
                                         ((8, 96, 16, 52), True), ((3, 100, 5, 9), False),
                                         ((4, 512, 4, 13), True)])
def test_corr_fwd_small_and_split_vs_tiled_and_oracle(hip_device, shape, split):
    """Small levels: the small-image kernel (one workgroup per sample, dy and
    row block, all channels staged at once; usf_corr_fwd_workspace == 0) or,
    where its rows do not fit the 32 KB stage, the channel split with its reduce
    (workspace > 0). Either matches the tiled kernel (variant 4, <4,4,8,3,8>)
    and the fp64 oracle; with the LeakyReLU epilogue into a concat slice it
    matches the composition, and its sign mask equals the tiled kernel's."""
    from unsamflow_amd import _lib, ops

    B, C, H, W = shape
    lib = _lib.load()
    assert (lib.usf_corr_fwd_workspace(B, C, H, W, 4) > 0) == split
    x1 = hashrng.normal(shape, 5 + C)
    x2 = hashrng.normal(shape, 6 + C)
    t1, t2 = _dev(x1, hip_device), _dev(x2, hip_device)
    small = ops.corr_forward(t1, t2, 4)
    cat = torch.full((B, 81 + 7, H, W), 7.0, device=hip_device)
    mask = ops.corr_act_mask(B, H, W, 4, hip_device)
    ops.corr_forward_ex(t1, t2, 4, cat[:, 3:84], leaky_slope=0.1, act_mask=mask)
    lib.usf_set_variant(0, 4)
    try:
        tiled = ops.corr_forward(t1, t2, 4)
        tmask = ops.corr_act_mask(B, H, W, 4, hip_device)
        tcat = torch.empty((B, 81, H, W), device=hip_device)
        ops.corr_forward_ex(t1, t2, 4, tcat, leaky_slope=0.1, act_mask=tmask)
    finally:
        lib.usf_set_variant(0, -1)
    ref = corr_forward_np(x1, x2, 4)
    np.testing.assert_allclose(_np(small), ref, atol=CORR_ATOL, rtol=CORR_RTOL)
    np.testing.assert_allclose(_np(small), _np(tiled), atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(_np(cat[:, 3:84]), _np(torch.nn.functional.leaky_relu(small, 0.1)), atol=0, rtol=0)
    assert float(cat[:, :3].min()) == 7.0 and float(cat[:, 84:].max()) == 7.0
    # the mask bits are the signs of this call's own outputs; the tiled kernel's
    # differ only where the two sums straddle zero
    pos = (cat[:, 3:84] > 0).reshape(B, 9, 9, H, W).cpu().numpy()
    bits = np.zeros((B, 9, H, (W + 3) // 4), np.uint64)
    for dx in range(9):
        for x in range(W):
            bits[..., x // 4] |= pos[:, :, dx, :, x].astype(np.uint64) << np.uint64(4 * dx + x % 4)
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), bits)
    tm = tmask.cpu().numpy().view(np.uint64)
    assert np.mean(tm == bits) > 0.99


@pytest.mark.parametrize("shape,scale", [((2, 8, 64, 208), 1.5), ((1, 4, 65, 130), 3.0), ((2, 4, 64, 208), 0.0)])
def test_warp_backward_default_large_levels(hip_device, shape, scale):
    """The default backward at large levels (the pixel-pair scatter: >= 4096 pairs
    per sample) against the oracle, incl. an odd height and zero flow (every pair
    merges)."""
    from unsamflow_amd import ops

    x = hashrng.uniform(shape, 600)
    flow = hashrng.symmetric((shape[0], 2) + shape[2:], 601, scale) if scale else \
        np.zeros((shape[0], 2) + shape[2:], np.float32)
    g = hashrng.normal(shape, 602)
    for pad in ("border", "zeros"):
        gx, gf = ops.warp_backward(_dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device), pad)
        rx, rf = warp_backward_np(x, flow, g, pad)
        np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
        np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("pad", ["border", "zeros"])
def test_warp_binned_gather_deterministic_and_overflow(hip_device, pad):
    """The default grad_x (binned gather, usf_warp_bwd_ex_f32): bit-identical
    across runs for a smooth flow (no cell holds more than 4 source pixels), and
    oracle-exact where most pixels overflow their cell (a flow contracting
    every pixel towards the image centre, so whole regions share a cell and the
    atomic overflow pass carries them)."""
    from unsamflow_amd import ops

    B, C, H, W = 2, 8, 40, 64
    x = hashrng.uniform((B, C, H, W), 700)
    g = hashrng.normal((B, C, H, W), 701)
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    smooth = np.stack([1.7 * np.sin(xx / 9.0) + 0.3, 1.2 * np.cos(yy / 7.0) - 0.4])[None].repeat(B, 0)
    contract = np.stack([0.9 * ((W - 1) / 2.0 - xx), 0.9 * ((H - 1) / 2.0 - yy)])[None].repeat(B, 0)
    for flow, deterministic in ((smooth.astype(np.float32), True), (contract.astype(np.float32), False)):
        tx, tf, tg = _dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device)
        gx, gf = ops.warp_backward(tx, tf, tg, pad)
        rx, rf = warp_backward_np(x, flow, g, pad)
        np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
        np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)
        if deterministic:
            gx2, _ = ops.warp_backward(tx, tf, tg, pad)
            assert torch.equal(gx, gx2)


def test_warp_bwd_plain_entry_is_the_scatter(hip_device):
    """usf_warp_bwd_f32 (no workspace) keeps the atomic scatter and matches the oracle."""
    from unsamflow_amd import _lib

    lib = _lib.load()
    shape = (2, 16, 24, 40)
    x = hashrng.uniform(shape, 710)
    flow = hashrng.symmetric((2, 2, 24, 40), 711, 3.0)
    g = hashrng.normal(shape, 712)
    tx, tf, tg = _dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device)
    gx, gf = torch.empty_like(tx), torch.empty(2, 2, 24, 40, device=hip_device)
    rc = lib.usf_warp_bwd_f32(tx.data_ptr(), tf.data_ptr(), 2 * 24 * 40, tg.data_ptr(), gx.data_ptr(),
                              gf.data_ptr(), *shape, _lib.PAD_BORDER, _lib.stream_handle(hip_device))
    _lib.check(rc, "usf_warp_bwd_f32")
    rx, rf = warp_backward_np(x, flow, g, "border")
    np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)


def _small_fields(B, H, W, kind):
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    if kind == "zero":
        f = np.zeros((2, H, W), np.float32)
    elif kind == "smooth":
        f = np.stack([1.7 * np.sin(xx / 3.0) + 0.3, 1.2 * np.cos(yy / 2.0) - 0.4])
    elif kind == "collapse":  # every pixel lands near one spot: cells with far more than 8 sources
        f = np.stack([0.95 * ((W - 1) / 2.0 - xx) + 0.3, 0.95 * ((H - 1) / 2.0 - yy) + 0.2])
    else:  # large random displacements, many off the image
        return hashrng.symmetric((B, 2, H, W), 733, 6.0)
    return np.ascontiguousarray(f[None].repeat(B, 0).astype(np.float32))


@pytest.mark.parametrize("pad", ["border", "zeros"])
@pytest.mark.parametrize("kind", ["zero", "smooth", "collapse", "random"])
@pytest.mark.parametrize("shape", [(4, 128, 8, 26), (3, 5, 7, 9), (2, 3, 16, 16)])
def test_warp_backward_small_image_vs_oracle(hip_device, shape, kind, pad):
    """The default backward on images of at most 256 pixels (the decoder's
    level 1 and smaller): matches the oracle for smooth, zero, fully
    contracting (cells with many sources: overflow entries) and large random
    flows; bit-identical across runs where no cell overflows (zero flow);
    each gradient alone equals its share of the joint call."""
    _small_image_case(hip_device, shape, kind, pad)


def _small_image_case(hip_device, shape, kind, pad):
    from unsamflow_amd import ops

    B, C, H, W = shape
    x = hashrng.uniform(shape, 730 + C)
    g = hashrng.normal(shape, 731 + C)
    flow = _small_fields(B, H, W, kind)
    tx, tf, tg = _dev(x, hip_device), _dev(flow, hip_device), _dev(g, hip_device)
    gx, gf = ops.warp_backward(tx, tf, tg, pad)
    rx, rf = warp_backward_np(x, flow, g, pad)
    np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)
    gx2, gf2 = ops.warp_backward(tx, tf, tg, pad)
    assert torch.equal(gf, gf2)
    if kind == "zero":  # no cell overflows: fixed-order sums only (this "smooth" field piles
        assert torch.equal(gx, gx2)  # border-clamped sources onto edge cells of these tiny images)
    else:
        torch.testing.assert_close(gx, gx2, atol=1e-5, rtol=1e-5)
    ox, _ = ops.warp_backward(tx, tf, tg, pad, need_flow=False)
    _, of = ops.warp_backward(tx, tf, tg, pad, need_x=False)
    torch.testing.assert_close(ox, gx, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(of, gf, atol=1e-5, rtol=1e-5)


def test_warp_backward_small_image_flow_slice(hip_device):
    """The loss-style flow slice (batch stride 4HW) through the backward at a small image."""
    from unsamflow_amd import ops

    B, C, H, W = 3, 16, 8, 26
    x = hashrng.uniform((B, C, H, W), 740)
    g = hashrng.normal((B, C, H, W), 741)
    f4 = hashrng.symmetric((B, 4, H, W), 742, 2.5)
    t4 = _dev(f4, hip_device)
    gx, gf = ops.warp_backward(_dev(x, hip_device), t4[:, 2:], _dev(g, hip_device), "border")
    rx, rf = warp_backward_np(x, np.ascontiguousarray(f4[:, 2:]), g, "border")
    np.testing.assert_allclose(_np(gx), rx, atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(_np(gf), rf, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("d", [1, 2, 3])
@pytest.mark.parametrize("shape", [(4, 64, 4, 13), (3, 48, 6, 26), (2, 40, 5, 10)])
def test_corr_fwd_small_kernel_every_d_vs_oracle(hip_device, d, shape):
    """fwd_plan sends the small levels to the small-image kernel for every d in
    1..4; its staging (V = 1 / 2 column pairs, HALO = 4 or 8, the window
    offsets) differs with d and with W's parity (advisor r03). Forward, the
    LeakyReLU epilogue and its sign mask against the fp64 oracle."""
    from unsamflow_amd import _lib, ops

    B, C, H, W = shape
    K = 2 * d + 1
    lib = _lib.load()
    assert lib.usf_corr_fwd_workspace(B, C, H, W, d) == 0  # the small kernel, not the split
    x1 = hashrng.normal(shape, 70 + d)
    x2 = hashrng.normal(shape, 80 + d)
    t1, t2 = _dev(x1, hip_device), _dev(x2, hip_device)
    ref = corr_forward_np(x1, x2, d)
    np.testing.assert_allclose(_np(ops.corr_forward(t1, t2, d)), ref, atol=CORR_ATOL, rtol=CORR_RTOL)
    cat = torch.full((B, K * K + 2, H, W), 7.0, device=hip_device)
    mask = ops.corr_act_mask(B, H, W, d, hip_device)
    ops.corr_forward_ex(t1, t2, d, cat[:, 1:1 + K * K], leaky_slope=0.1, act_mask=mask)
    act = np.where(ref > 0, ref, ref * np.float32(0.1))
    np.testing.assert_allclose(_np(cat[:, 1:1 + K * K]), act, atol=CORR_ATOL, rtol=CORR_RTOL)
    assert float(cat[:, 0].min()) == 7.0 and float(cat[:, -1].max()) == 7.0
    if mask is not None:
        pos = (cat[:, 1:1 + K * K] > 0).reshape(B, K, K, H, W).cpu().numpy()
        bits = np.zeros((B, K, H, (W + 3) // 4), np.uint64)
        for dx in range(K):
            for x in range(W):
                bits[..., x // 4] |= pos[:, :, dx, :, x].astype(np.uint64) << np.uint64(4 * dx + x % 4)
        assert np.array_equal(mask.cpu().numpy().view(np.uint64), bits)

