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
