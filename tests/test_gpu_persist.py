"""The persistent forms (ABI 7): usf_warp_bwd_persist_f32
(binned gather without the per-call zero fill: two launches with a dense
overflow buffer up to 8192 pixels, three -- the overflow pass kept -- in the
list form above) and usf_occ_backward_persist_f32 (splat + threshold, the
threshold re-zeroes the splat buffer). Their workspaces carry state from one
call to the next, so every test runs a SEQUENCE of calls on one workspace --
overflow-heavy, then smooth, then overflow-heavy again, and a second shape in
between -- and checks each against the per-call forms (usf_warp_bwd_ex_f32,
usf_occ_backward_f32), which zero their state on every call:
grad_flow bit-identical, grad_x bit-identical where no cell overflows and
within atol 1e-5 where overflow entries are summed by fp32 atomics
(utils/warp_utils.py:97-106 / :120-126 via the reference-pinned per-call forms).
"""
import pytest
import torch

from unsamflow_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _fields(B, H, W, dev):
    yy = torch.arange(H, device=dev, dtype=torch.float32).view(1, H, 1).expand(1, H, W)
    xx = torch.arange(W, device=dev, dtype=torch.float32).view(1, 1, W).expand(1, H, W)
    smooth = torch.cat([1.7 * torch.sin(xx / 9.0) + 0.3, 1.2 * torch.cos(yy / 7.0) - 0.4]).expand(B, 2, H, W)
    shift = smooth.clone()
    shift[:, 0] += W / 8.0  # border-clamped strip: many sources on one edge cell per row (overflow)
    contract = torch.cat([0.9 * ((W - 1) / 2.0 - xx), 0.9 * ((H - 1) / 2.0 - yy)]).expand(B, 2, H, W)
    return {"smooth": smooth.contiguous(), "shift": shift.contiguous(), "contract": contract.contiguous()}


def _ex(x, flow, go, pad):
    """usf_warp_bwd_ex_f32: the four-launch form with a fresh workspace (zero-filled by the call)."""
    lib = _lib.load()
    B, C, H, W = x.shape
    gx, gf = torch.empty_like(x), torch.empty(B, 2, H, W, device=x.device)
    n = int(lib.usf_warp_bwd_workspace(B, H, W))
    ws = torch.empty(n, device=x.device, dtype=torch.uint8)
    rc = lib.usf_warp_bwd_ex_f32(x.data_ptr(), flow.data_ptr(), 2 * H * W, go.data_ptr(), gx.data_ptr(),
                                 gf.data_ptr(), ws.data_ptr(), n, B, C, H, W,
                                 _lib.PAD_BORDER if pad == "border" else _lib.PAD_ZEROS,
                                 _lib.stream_handle(x.device))
    _lib.check(rc, "usf_warp_bwd_ex_f32")
    return gx, gf


@pytest.mark.parametrize("pad", ["border", "zeros"])
def test_warp_persist_call_sequence_matches_per_call_form(hip_device, pad, monkeypatch):
    monkeypatch.setattr(ops, "WARP_PERSIST_MAX_PIXELS", None)  # the persistent form at every shape
    shapes = [(4, 32, 64, 208), (3, 16, 33, 70)]
    data = {}
    for i, (B, C, H, W) in enumerate(shapes):
        g = torch.Generator(device=hip_device).manual_seed(20 + i)
        data[(B, C, H, W)] = (torch.randn(B, C, H, W, device=hip_device, generator=g),
                              torch.randn(B, C, H, W, device=hip_device, generator=g),
                              _fields(B, H, W, hip_device))
    seq = [(0, "shift"), (0, "smooth"), (1, "contract"), (0, "contract"), (0, "smooth"), (1, "smooth"),
           (0, "shift"), (1, "shift"), (0, "smooth")]
    for si, kind in seq:
        x, go, fields = data[shapes[si]]
        flow = fields[kind]
        gx, gf = ops.warp_backward(x, flow, go, pad, True, True)  # the persistent form
        rx, rf = _ex(x, flow, go, pad)
        assert torch.equal(gf, rf), (shapes[si], kind)
        if kind == "smooth":
            assert torch.equal(gx, rx), (shapes[si], kind)  # no overflow: the same fixed-order sums
        else:
            torch.testing.assert_close(gx, rx, atol=1e-5, rtol=1e-5, msg=lambda m: f"{shapes[si]} {kind}: {m}")


def test_warp_persist_workspace_returns_to_reusable_state(hip_device, monkeypatch):
    """After an overflow-heavy call and a smooth one, the workspace holds no
    leftover: the overflow buffer and every dirty word are zero again, and one
    of the two count buffers is zero (the one the next call files into)."""
    monkeypatch.setattr(ops, "WARP_PERSIST_MAX_PIXELS", None)
    B, C, H, W = 2, 16, 40, 64
    g = torch.Generator(device=hip_device).manual_seed(31)
    x = torch.randn(B, C, H, W, device=hip_device, generator=g)
    go = torch.randn(B, C, H, W, device=hip_device, generator=g)
    f = _fields(B, H, W, hip_device)
    ops.warp_backward(x, f["contract"], go, "border")
    ops.warp_backward(x, f["smooth"], go, "border")
    torch.cuda.synchronize()
    ws = ops.persistent_workspace(hip_device, "warp_bwd", (B, C, H, W), 0)
    # layout of warp.hip bin_layout2, restated: header, 2 count buffers, slots, weights, dirty words, overflow
    al = lambda v: (v + 255) & ~255  # noqa: E731
    cells = B * (H + 1) * (W + 1)
    ntiles = ((W + 31) // 32) * ((H + 7) // 8)
    bins_off = al(256 + 8 * cells)
    dirty_off = al(al(bins_off + 16 * cells) + 64 * cells)
    total = al(al(dirty_off + 4 * B * ntiles) + 4 * B * C * H * W)
    assert total == int(_lib.load().usf_warp_bwd_persist_workspace(B, C, H, W)) <= ws.numel()
    assert int(torch.count_nonzero(ws[dirty_off:total])) == 0  # dirty words and the overflow buffer
    hdr = ws[:8].view(torch.int32).cpu()
    cnt = ws[256:256 + 8 * cells].view(torch.int32).view(2, cells)
    nxt = int(hdr[0])
    assert nxt in (0, 1) and int(torch.count_nonzero(cnt[nxt])) == 0


def test_warp_persist_list_form_returns_to_reusable_state(hip_device, monkeypatch):
    """The list form (levels above USF_PERSIST_LIST_PIXELS = 8192 pixels: filing,
    gather, overflow pass; no zero fill): after an overflow-heavy call and a
    smooth one, the count buffer and the list length the parity selects for the
    next call are zero, and every call matched the per-call form."""
    monkeypatch.setattr(ops, "WARP_PERSIST_MAX_PIXELS", None)
    B, C, H, W = 2, 8, 96, 100
    g = torch.Generator(device=hip_device).manual_seed(37)
    x = torch.randn(B, C, H, W, device=hip_device, generator=g)
    go = torch.randn(B, C, H, W, device=hip_device, generator=g)
    f = _fields(B, H, W, hip_device)
    for kind in ("contract", "shift", "smooth", "contract", "smooth"):
        gx, gf = ops.warp_backward(x, f[kind], go, "border")
        rx, rf = _ex(x, f[kind], go, "border")
        assert torch.equal(gf, rf), kind
        if kind == "smooth":
            assert torch.equal(gx, rx), kind
        else:
            torch.testing.assert_close(gx, rx, atol=1e-5, rtol=1e-5)
    torch.cuda.synchronize()
    ws = ops.persistent_workspace(hip_device, "warp_bwd", (B, C, H, W), 0)
    # bin_layout2's list form, restated: header, 2 count buffers, slots, weights, overflow list
    al = lambda v: (v + 255) & ~255  # noqa: E731
    cells = B * (H + 1) * (W + 1)
    ovf_off = al(al(al(256 + 8 * cells) + 16 * cells) + 64 * cells)
    assert al(ovf_off + 4 * B * H * W) == int(_lib.load().usf_warp_bwd_persist_workspace(B, C, H, W))
    hdr = ws[:16].view(torch.int32).cpu()
    cnt = ws[256:256 + 8 * cells].view(torch.int32).view(2, cells)
    nxt = int(hdr[0])
    assert nxt in (0, 1) and int(torch.count_nonzero(cnt[nxt])) == 0 and int(hdr[2 + nxt]) == 0


def test_occ_persist_call_sequence_matches_per_call_form(hip_device):
    lib = _lib.load()
    for B, H, W in [(8, 256, 832), (2, 40, 64), (8, 256, 832)]:
        f = _fields(B, H, W, hip_device)
        for kind in ("smooth", "contract", "shift", "smooth"):
            flow = f[kind]
            got = ops.occ_backward(flow, 0.2)  # the persistent form
            ref = torch.empty_like(got)
            rc = lib.usf_occ_backward_f32(flow.data_ptr(), 2 * H * W, ref.data_ptr(), B, H, W, 0.2,
                                          _lib.stream_handle(hip_device))
            _lib.check(rc, "usf_occ_backward_f32")
            # masks agree except where the splat sum sits within 1e-5 of the threshold
            # (atomic summation order, as in tests/test_gpu_parity.py's occlusion checks)
            diff = (got != ref)
            if diff.any():
                m = torch.empty_like(got)
                rc = lib.usf_splat_map_f32(flow.data_ptr(), 2 * H * W, m.data_ptr(), B, H, W, 0,
                                           _lib.stream_handle(hip_device))
                _lib.check(rc, "usf_splat_map_f32")
                assert bool(((m[diff].clamp(0, 1) - 0.2).abs() < 1e-5).all()), (B, H, W, kind)
    torch.cuda.synchronize()
    for key, (ws, _) in ops._PERSIST.items():
        if key[1] == "occ_bwd":
            assert int(torch.count_nonzero(ws)) == 0, key  # the threshold pass left every map zero


def _np_fields(B, H, W):
    """Decoder-style flows as numpy: a smooth +-2 px field with a per-sample
    phase, a border-piling shift (a strip of sources clamped onto the edge
    column: many pixels per cell), and a field contracting towards the centre
    (whole regions share a cell: overflow entries and dirty tiles)."""
    import numpy as np

    yy, xx = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    ph = np.arange(B, dtype=np.float32).reshape(B, 1, 1) * 0.7
    u = np.sin(2 * np.pi * 2 * xx / W + ph) + np.cos(2 * np.pi * 3 * yy / H - ph)
    v = np.cos(2 * np.pi * 2 * xx / W - ph) - np.sin(2 * np.pi * 3 * yy / H + ph)
    smooth = np.stack([u, v], 1).astype(np.float32)
    pile = smooth.copy()
    pile[:, 0] += W / 8.0
    contract = np.stack([0.9 * ((W - 1) / 2.0 - xx), 0.9 * ((H - 1) / 2.0 - yy)])[None].repeat(B, 0)
    return {"smooth": smooth, "pile": pile, "contract": contract.astype(np.float32)}


@pytest.mark.parametrize("form", ["production", "persist"])
@pytest.mark.parametrize("pad", ["border", "zeros"])
@pytest.mark.parametrize("shape", [(16, 128, 8, 26), (16, 96, 16, 52), (16, 64, 32, 104), (16, 32, 64, 208)])
def test_warp_persist_production_shapes_vs_oracle(hip_device, shape, pad, form, monkeypatch):
    """the warp backward at the decoder's four warp sites at
    batch 16 against the CPU oracle (oracle/warp.py, restating
    utils/warp_utils.py:97-106 + ATen's sampler), as a call SEQUENCE on one
    workspace: smooth, border-piling, contracting, smooth again. ``persist``
    forces the persistent two-launch form (usf_warp_bwd_persist_f32, whose
    workspace carries a parity word, dirty-tile marks and an overflow buffer
    from call to call) at every level; ``production`` is ops.warp_backward's
    own choice per level (ops.WARP_PERSIST_MAX_PIXELS). Tolerances of SURVEY
    8(c): grad_x and grad_flow atol 1e-4, rtol 1e-5."""
    import numpy as np

    from oracle import hashrng
    from oracle.warp import warp_backward_np

    if form == "persist":
        monkeypatch.setattr(ops, "WARP_PERSIST_MAX_PIXELS", None)
    B, C, H, W = shape
    x = hashrng.uniform(shape, 900 + C)
    g = hashrng.normal(shape, 901 + C)
    tx, tg = torch.from_numpy(x).to(hip_device), torch.from_numpy(g).to(hip_device)
    fields = _np_fields(B, H, W)
    ops.clear_persistent_workspaces()
    for kind in ("smooth", "pile", "contract", "smooth"):
        flow = fields[kind]
        gx, gf = ops.warp_backward(tx, torch.from_numpy(flow).to(hip_device), tg, pad, True, True)
        rx, rf = warp_backward_np(x, flow, g, pad)
        np.testing.assert_allclose(gx.cpu().numpy(), rx, atol=1e-4, rtol=1e-5, err_msg=f"{shape} {pad} {kind} gx")
        np.testing.assert_allclose(gf.cpu().numpy(), rf, atol=1e-4, rtol=1e-5, err_msg=f"{shape} {pad} {kind} gflow")
    persisted = (hip_device.index, "warp_bwd", shape) in ops._PERSIST
    assert persisted == (form == "persist" or ops.WARP_PERSIST_MAX_PIXELS is None or H * W <= ops.WARP_PERSIST_MAX_PIXELS)


def test_persistent_workspace_cache_is_bounded_and_ordered(hip_device, monkeypatch):
    """the cache keeps at most PERSIST_MAX_ENTRIES shapes (least
    recently used out), and a use from another stream is ordered after the
    previous one (the new stream waits for the owning stream)."""
    monkeypatch.setattr(ops, "WARP_PERSIST_MAX_PIXELS", None)
    ops.clear_persistent_workspaces()
    for i in range(ops.PERSIST_MAX_ENTRIES + 5):
        ops.persistent_workspace(hip_device, "test_op", (i,), 64)
    keys = [k for k in ops._PERSIST if k[1] == "test_op"]
    assert len(keys) == ops.PERSIST_MAX_ENTRIES and keys[0][2] == (5,)
    # a warp call on a side stream right after one on the main stream gives the same result
    B, C, H, W = 2, 16, 40, 64
    gen = torch.Generator(device=hip_device).manual_seed(5)
    x = torch.randn(B, C, H, W, device=hip_device, generator=gen)
    go = torch.randn(B, C, H, W, device=hip_device, generator=gen)
    f = _fields(B, H, W, hip_device)
    ref = ops.warp_backward(x, f["contract"], go, "border")
    side = torch.cuda.Stream(hip_device)
    side.wait_stream(torch.cuda.current_stream(hip_device))
    with torch.cuda.stream(side):
        a = ops.warp_backward(x, f["contract"], go, "border")
        assert ops._PERSIST[(hip_device.index, "warp_bwd", (B, C, H, W))][1] == side
    b = ops.warp_backward(x, f["contract"], go, "border")  # main stream again: waits for the side stream
    torch.cuda.synchronize()
    for r, s1, s2 in zip(ref, a, b):
        torch.testing.assert_close(s1, r, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(s2, r, atol=1e-5, rtol=1e-5)
    ops.clear_persistent_workspaces()


@pytest.mark.parametrize("pad", ["border", "zeros"])
def test_warp_small_fused_is_deterministic_and_matches_oracle(hip_device, pad):
    """Small levels (H*W <= 512: KITTI L1, Sintel L1) take one fused launch that
    bins every sample's pixels in LDS and sums each cell's pixels in index
    order: no overflow atomics, so grad_x is bit-identical from call to call
    even where cells hold many pixels, and both grads match the oracle
    (utils/warp_utils.py:97-106; tolerances of SURVEY 8(c))."""
    import numpy as np

    from oracle import hashrng
    from oracle.warp import warp_backward_np

    B, C, H, W = 4, 24, 12, 20
    x = hashrng.uniform((B, C, H, W), 950)
    g = hashrng.normal((B, C, H, W), 951)
    tx, tg = torch.from_numpy(x).to(hip_device), torch.from_numpy(g).to(hip_device)
    fields = _np_fields(B, H, W)
    for kind in ("contract", "pile", "smooth"):
        flow = torch.from_numpy(fields[kind]).to(hip_device)
        gx1, gf1 = ops.warp_backward(tx, flow, tg, pad, True, True)
        gx2, gf2 = ops.warp_backward(tx, flow, tg, pad, True, True)
        assert torch.equal(gx1, gx2) and torch.equal(gf1, gf2), kind
        rx, rf = warp_backward_np(x, fields[kind], g, pad)
        np.testing.assert_allclose(gx1.cpu().numpy(), rx, atol=1e-4, rtol=1e-5, err_msg=f"{pad} {kind} gx")
        np.testing.assert_allclose(gf1.cpu().numpy(), rf, atol=1e-4, rtol=1e-5, err_msg=f"{pad} {kind} gflow")
