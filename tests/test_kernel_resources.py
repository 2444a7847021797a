"""Register / LDS budgets of the gfx950 kernels (compile-only, no GPU).

The correlation kernels are latency-bound at PWCLite's shapes, so their speed
rests on occupancy: the default backward tile <d=4, PX=4, SEGX=8, NW=3, CC=4>
must stay within 168 VGPRs (3 waves/SIMD) and 40 KB of LDS (4 workgroups of
3 waves per CU), and no kernel may spill to scratch.
"""
import re
import shutil

import pytest

from conftest import REPO

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")


@pytest.fixture(scope="module")
def corr_resources():
    import sys

    sys.path.insert(0, str(REPO / "tools"))
    import kernel_resources

    return kernel_resources.resources(REPO / "unsamflow_amd" / "csrc" / "corr.hip")


def test_no_kernel_spills(corr_resources):
    spilled = [(n, s) for n, _, _, s in corr_resources if s]
    assert not spilled, spilled


def test_default_backward_tile_occupancy(corr_resources):
    # <4,4,8,3,4, V, MODE, AM, NB = 2>
    default = [r for r in corr_resources if re.search(r"corr_bwd_kernelILi4ELi4ELi8ELi3ELi4ELi\dELi\dELb\dELi2E", r[0])]
    assert default, "default backward instantiation missing"
    for name, vgpr, lds, _ in default:
        assert vgpr <= 168, (name, vgpr)
        assert lds <= 40 * 1024, (name, lds)


def test_large_level_forward_occupancy(corr_resources):
    """The L3/L4 forward tile <d=4, PX=4, SEGX=8, NDY=9, CC=4> keeps its 7
    waves/SIMD with the sign-mask epilogue (a per-bit bounds test in the
    epilogue once raised it from 65 to 101 VGPRs and slowed L4 by ~25%)."""
    # <4,4,8,9,4, V, CS = 1>
    fwd = [r for r in corr_resources if re.search(r"corr_fwd_kernelILi4ELi4ELi8ELi9ELi4ELi\dELi1EE", r[0])]
    assert fwd, "large-level forward instantiation missing"
    for name, vgpr, _, _ in fwd:
        assert vgpr <= 72, (name, vgpr)


def _hazard_tool():
    import sys

    sys.path.insert(0, str(REPO / "tools"))
    import lds_dma_hazard

    return lds_dma_hazard


def test_every_lds_dma_in_the_built_library_is_guarded():
    """every buffer_load_dword{,x4} ... lds of the library's
    gfx950 code objects sits behind s_nop >= 4 (or 5 straight-line wait states
    with no VALU write of an SGPR it reads) -- the hazard that faulted a box in
    round 4 is caught here, at build time."""
    from unsamflow_amd.build import LIB_PATH, build_library

    build_library()
    n, bad = _hazard_tool().check_library(LIB_PATH)
    assert n > 1000, f"expected the correlation kernels' LDS-DMA sites, found {n}"
    assert not bad, bad[:5]


def test_lds_dma_hazard_checker_flags_an_unpadded_dma():
    t = _hazard_tool()
    dma = (0x20, "buffer_load_dwordx4", "v8, s[16:19], 0 offen lds")
    unpadded = [(0x10, "v_readlane_b32", "s17, v40, 3"), (0x18, "s_mov_b32", "m0, s0"), dma]
    padded = unpadded[:2] + [(0x1C, "s_nop", "4"), dma]
    far = [(0x0, "v_readfirstlane_b32", "s16, v1")] + [(0x4 + 4 * i, "s_add_u32", "s2, s2, 1") for i in range(5)] \
        + [(0x20, dma[1], dma[2])]
    assert t.analyze(unpadded)[1] and not t.analyze(padded)[1] and not t.analyze(far)[1]
    # a branch landing between the SGPR write and the DMA voids the straight-line argument
    branchy = [(0x0, "v_readfirstlane_b32", "s16, v1"), (0x4, "s_cbranch_scc1", "2"), (0x8, "s_nop", "0"),
               (0xC, "s_nop", "0"), (0x10, "s_add_u32", "s2, s2, 1"), (0x14, "s_add_u32", "s2, s2, 1"),
               (0x18, dma[1], dma[2])]
    assert t.analyze(branchy)[1]
