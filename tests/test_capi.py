"""C-ABI boundary checks that need no GPU: the library loads, exports exactly
what include/unsamflow_hip.h declares, reports its ABI version, and rejects bad
arguments with USF_EINVAL + an error string before touching the device."""
import ctypes
import re
import subprocess

import pytest

from conftest import REPO

HEADER = REPO / "include" / "unsamflow_hip.h"


@pytest.fixture(scope="module")
def lib():
    from unsamflow_amd import _lib
    from unsamflow_amd.build import build_library

    build_library()
    return _lib.load()


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(usf_\w+)\s*\(", text)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert syms == sorted(
        ["usf_abi_version", "usf_build_id", "usf_last_error_string", "usf_corr_fwd_f32", "usf_corr_bwd_f32",
         "usf_corr_fwd_ex_f32", "usf_corr_fwd_workspace", "usf_corr_bwd_ex_f32", "usf_corr_act_mask_words",
         "usf_corr_bwd_ex_scratch",
         "usf_warp_fwd_f32", "usf_warp_fwd_up_f32", "usf_warp_bwd_f32", "usf_warp_bwd_ex_f32", "usf_warp_bwd_workspace",
         "usf_warp_bwd_persist_f32", "usf_warp_bwd_persist_workspace",
         "usf_splat_map_f32", "usf_occ_backward_f32", "usf_occ_backward_persist_f32", "usf_occ_vis_pair_persist_f32",
         "usf_occ_bidirection_f32",
         "usf_photo_loss_partials", "usf_photo_loss_fwd_f32", "usf_photo_loss_pair_fwd_f32",
         "usf_photo_loss_bwd_f32", "usf_photo_loss_pyramid_partials", "usf_photo_loss_pyramid_fwd_f32",
         "usf_photo_loss_pyramid_bwd_f32",
         "usf_flow_upsample_f32", "usf_flow_upsample_bwd_f32", "usf_flow_upsample_bwd_sum_f32", "usf_area_pyramid_f32",
         "usf_convex_upsample_f32", "usf_convex_upsample_bwd_scratch", "usf_convex_upsample_bwd_f32",
         "usf_convex_upsample_pyramid_f32", "usf_convex_upsample_pyramid_bwd_scratch",
         "usf_convex_upsample_pyramid_bwd_f32",
         "usf_set_variant", "usf_device_errors", "usf_stream_copy_f32"]
    )


def test_library_exports_every_declared_symbol(lib):
    from unsamflow_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.library_path())], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (usf_\w+)", out))
    for s in declared_symbols():
        assert s in exported, s
        assert hasattr(lib, s)
    assert set(_lib.EXPORTED_SYMBOLS) == set(declared_symbols())


def test_build_id_matches_the_tree(lib):
    """The library carries the id of the sources it was built from, so a
    measurement summary can be matched to the build it was taken on."""
    from unsamflow_amd import _lib
    from unsamflow_amd.build import build_id

    assert _lib.build_id() == build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", _lib.build_id())


def test_abi_version(lib):
    from unsamflow_amd import _lib

    assert lib.usf_abi_version() == _lib.ABI_VERSION == 8


def test_no_torch_types_in_abi():
    text = HEADER.read_text()
    for bad in ("at::", "torch", "Tensor", "c10"):
        # the header only mentions torch in prose comments
        code = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        assert bad not in code


@pytest.mark.parametrize(
    "call,needle",
    [
        (lambda L: L.usf_corr_fwd_f32(1, 1, 1, 0, 4, 4, 4, 4, None), "non-positive shape"),
        (lambda L: L.usf_corr_fwd_f32(1, 1, 1, 1, 4, 4, 4, 5, None), "max_displacement 5"),
        (lambda L: L.usf_corr_fwd_f32(None, 1, 1, 1, 4, 4, 4, 4, None), "null pointer"),
        (lambda L: L.usf_corr_bwd_f32(1, 1, None, 1, 1, 1, 4, 4, 4, 4, None), "null input"),
        (lambda L: L.usf_corr_bwd_f32(1, 1, 1, 1, 1, 1, 4, 4, 4, 0, None), "max_displacement 0"),
        (lambda L: L.usf_warp_fwd_f32(1, 1, 32, 1, 1, 3, 4, 4, 7, None), "pad_mode 7"),
        (lambda L: L.usf_warp_fwd_f32(1, 1, 3, 1, 2, 3, 4, 4, 1, None), "batch stride"),
        (lambda L: L.usf_warp_fwd_up_f32(1, 1, 1, 1, 2, 3, 5, 4, 1, None), "must be even"),
        (lambda L: L.usf_warp_fwd_up_f32(1, None, 1, 1, 2, 3, 4, 4, 1, None), "null pointer"),
        (lambda L: L.usf_warp_bwd_f32(1, None, 32, 1, 1, 1, 1, 3, 4, 4, 1, None), "null input"),
        (lambda L: L.usf_warp_bwd_f32(1, 1, 32, 1, 1, 1, 1, 3, -4, 4, 1, None), "non-positive"),
        (lambda L: L.usf_warp_bwd_ex_f32(1, 1, 32, 1, 1, 1, 1, -5, 1, 3, 4, 4, 1, None), "negative workspace"),
        (lambda L: L.usf_warp_bwd_ex_f32(1, 1, 32, 1, 1, 1, 1, 64, 1, 3, 4, 4, 5, None), "pad_mode 5"),
        (lambda L: L.usf_corr_fwd_f32(1, 1, 1, 1, 70000, 200, 200, 4, None), "too large"),
        (lambda L: L.usf_corr_fwd_ex_f32(1, 1, 1, 10, 1, 0.1, None, None, 0, 2, 4, 4, 4, 4, None), "out batch stride"),
        (lambda L: L.usf_corr_fwd_ex_f32(1, 1, 1, 81 * 16, 7, 0.1, None, None, 0, 2, 4, 4, 4, 4, None), "unknown act"),
        (lambda L: L.usf_corr_fwd_ex_f32(1, 1, 1, 81 * 16, 0, 0.1, 1, None, 0, 2, 4, 4, 4, 4, None), "act_mask needs"),
        (lambda L: L.usf_corr_bwd_ex_f32(1, 1, 1, 10, None, None, 0.1, None, 1, 1, 2, 4, 4, 4, 4, None), "gradient batch stride"),
        (lambda L: L.usf_corr_bwd_ex_f32(1, 1, 1, 81 * 20, 1, None, 0.1, None, 1, 1, 2, 4, 4, 5, 4, None), "scratch"),
        (lambda L: L.usf_flow_upsample_f32(1, 1, 1, 2, 4, 4, 0, None), "bad factor"),
        (lambda L: L.usf_flow_upsample_bwd_f32(None, 1, 1, 2, 4, 4, 2, None), "null pointer"),
        (lambda L: L.usf_flow_upsample_bwd_sum_f32(1, None, 1, 1, 2, 4, 4, 2, None), "null pointer"),
        (lambda L: L.usf_splat_map_f32(1, 2 * 16, 1, 0, 4, 4, 0, None), "non-positive"),
        (lambda L: L.usf_splat_map_f32(None, 2 * 16, 1, 1, 4, 4, 0, None), "null pointer"),
        (lambda L: L.usf_occ_backward_f32(1, 3, 1, 2, 4, 4, 0.2, None), "batch stride"),
        (lambda L: L.usf_occ_backward_f32(1, 32, None, 1, 4, 4, 0.2, None), "null pointer"),
        (lambda L: L.usf_occ_backward_persist_f32(1, 32, 16, 16, 60, 1, 4, 4, 0.2, None), "separate buffer"),
        (lambda L: L.usf_occ_backward_persist_f32(1, 32, 16, 16, 64, 1, 4, 4, 0.2, None), "separate buffer"),
        (lambda L: L.usf_warp_bwd_persist_f32(1, 1, 32, 1, 1, 1, 16, 64, 1, 3, 4, 4, 1, None), "persistent workspace"),
        (lambda L: L.usf_occ_vis_pair_persist_f32(1, 80, 16, 32, 1 << 20, 2, 4, 4, 0.2, None), "dense [B,4,H,W]"),
        (lambda L: L.usf_occ_vis_pair_persist_f32(1, 64, 16, 32, 100, 2, 4, 4, 0.2, None), "separate buffer"),
        (lambda L: L.usf_occ_vis_pair_persist_f32(1, 64, None, 32, 1 << 20, 2, 4, 4, 0.2, None), "null pointer"),
        (lambda L: L.usf_warp_bwd_persist_f32(1, 1, 32, 1, 1, 1, 16, 1 << 40, 1, 300, 4, 4, 1, None), "C=300"),
        # both count buffers of the persistent form must stay under 32-bit byte offsets
        (lambda L: L.usf_warp_bwd_persist_f32(1, 1, 8192, 1, 16, 1, 16, 1 << 60, 70000, 4, 64, 64, 1, None), "2^31"),
        (lambda L: L.usf_photo_loss_fwd_f32(1, 1, 1, 1, 32, 1, 1, None, 1, 4, 4, 4, 1, 0.15, 0.85, None), "> 3"),
        (lambda L: L.usf_photo_loss_fwd_f32(1, 1, 1, 1, 32, 1, 1, 1, 1, 3, 4, 4, 9, 0.15, 0.85, None), "pad_mode 9"),
        (lambda L: L.usf_photo_loss_fwd_f32(1, None, 1, 1, 32, 1, 1, None, 1, 3, 4, 4, 1, 0.15, 0.85, None), "null input"),
        (lambda L: L.usf_photo_loss_bwd_f32(1, None, 1, 1, 1, 4, 4, 1, None), "null pointer"),
        (lambda L: L.usf_photo_loss_pyramid_fwd_f32(5, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, None, 1, 3, 1, 0.15, 0.85,
                                                     None), "nscale 5"),
        (lambda L: L.usf_photo_loss_pyramid_bwd_f32(0, 1, 1, 1, 1, 1, 1, 1, None), "nscale 0"),
        (lambda L: L.usf_area_pyramid_f32(1, 1, 1, 1, 1, 3, 12, 16, None), "multiples of 8"),
        (lambda L: L.usf_area_pyramid_f32(1, None, 1, 1, 1, 3, 16, 16, None), "null pointer"),
        (lambda L: L.usf_photo_loss_bwd_f32(1, 1, 1, 1, 0, 4, 4, 1, None), "non-positive"),
        (lambda L: L.usf_photo_loss_bwd_f32(1, 1, 1, 1, 1, 4, 4, 3, None), "ndir=3"),
        (lambda L: L.usf_photo_loss_pair_fwd_f32(1, 1, 1, 1, 1, 32, 1, 1, None, 2, 3, 4, 4, 1, 0.15, 0.85, None), "< 4*H*W"),
        (lambda L: L.usf_convex_upsample_f32(1, 1, 1, 2, 4, 4, 3, 0.25, None), "factor 3"),
        (lambda L: L.usf_convex_upsample_f32(1, None, 1, 2, 4, 4, 4, 0.25, None), "null pointer"),
        (lambda L: L.usf_convex_upsample_f32(1, 1, 1, 2, 0, 4, 4, 0.25, None), "non-positive"),
        (lambda L: L.usf_convex_upsample_bwd_f32(1, 1, 1, 1, 1, None, 2, 4, 4, 4, 0.25, None), "needs scratch"),
        (lambda L: L.usf_convex_upsample_bwd_f32(1, 1, None, 1, 1, 1, 2, 4, 4, 4, 0.25, None), "null input"),
        (lambda L: L.usf_photo_loss_pair_fwd_f32(1, 1, 1, None, 1, 64, 1, 1, None, 2, 3, 4, 4, 1, 0.15, 0.85, None), "null input"),
    ],
)
def test_invalid_arguments_rejected_without_launch(lib, call, needle):
    rc = call(lib)
    assert rc == -1
    msg = lib.usf_last_error_string().decode()
    assert needle in msg, msg


def test_error_string_cleared_on_next_call(lib):
    assert lib.usf_corr_fwd_f32(1, 1, 1, 0, 4, 4, 4, 4, None) == -1
    assert lib.usf_last_error_string() != b""
    # a warp bwd with neither output requested is a valid no-op (no launch)
    assert lib.usf_warp_bwd_f32(1, 1, 32, 1, None, None, 1, 3, 4, 4, 1, None) == 0
    assert lib.usf_last_error_string() == b""


def test_variant_override_bounds(lib):
    n_fwd = lib.usf_set_variant(0, -1)
    n_bwd = lib.usf_set_variant(1, -1)
    assert n_fwd > 1 and n_bwd > 1
    assert lib.usf_set_variant(0, n_fwd) == -1 and b"bad op" in lib.usf_last_error_string()
    assert lib.usf_set_variant(4, 0) == -1
    assert lib.usf_set_variant(3, 0) == 1 and lib.usf_set_variant(3, -1) == 1  # photometric: the pair kernel only
    assert lib.usf_set_variant(3, 1) == -1
    assert lib.usf_set_variant(2, 1) == 3 and lib.usf_set_variant(2, -1) == 3  # warp grad_x: scatter, pairs, bins
    assert lib.usf_set_variant(1, n_bwd - 1) == n_bwd
    assert lib.usf_set_variant(1, -1) == n_bwd


def test_ctypes_signatures_match_header():
    """argtype counts of the ctypes binding equal the C prototypes' parameter counts."""
    from unsamflow_amd import _lib

    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    for name, (argtypes, _) in _lib._SIGNATURES.items():
        m = re.search(name + r"\s*\(([^)]*)\)", text)
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(argtypes), name
    assert ctypes.sizeof(ctypes.c_longlong) == 8


def test_warp_bwd_workspace_size(lib):
    """Workspace of the binned gather: counts, 4 slots (+ weights) per cell of the
    (H+1) x (W+1) grid, overflow list; 0 for a non-positive shape."""
    B, H, W = 16, 64, 208
    n = lib.usf_warp_bwd_workspace(B, H, W)
    cells = B * (H + 1) * (W + 1)
    assert 4 * cells * (1 + 4 + 16) + 4 * B * H * W <= n <= 4 * cells * (1 + 4 + 16) + 4 * B * H * W + 5 * 256
    assert lib.usf_warp_bwd_workspace(0, H, W) == 0


def test_warp_bwd_persist_workspace_size(lib):
    """Persistent form: two count buffers, 4 slots + weights per cell, then up
    to 8192 pixels a dirty word per gather tile and a dense [B,C,H,W] overflow
    buffer, above that an overflow list of one int per pixel; 0 when invalid."""
    B, C, H, W = 16, 32, 32, 104  # 3328 pixels: the dense overflow buffer
    n = lib.usf_warp_bwd_persist_workspace(B, C, H, W)
    cells = B * (H + 1) * (W + 1)
    lo = 4 * cells * (2 + 4 + 16) + 4 * B * C * H * W
    assert lo <= n <= lo + 4 * B * 4 * 4 + 6 * 256
    B, C, H, W = 16, 32, 64, 208  # 13312 pixels: the list form
    n = lib.usf_warp_bwd_persist_workspace(B, C, H, W)
    cells = B * (H + 1) * (W + 1)
    lo = 4 * cells * (2 + 4 + 16) + 4 * B * H * W
    assert lo <= n <= lo + 5 * 256
    assert lib.usf_warp_bwd_persist_workspace(B, 0, H, W) == 0
