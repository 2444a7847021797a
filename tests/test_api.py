"""Host-side API surface of the drop-ins (no GPU needed): constructor forms,
supported-subset checks, no parameters/buffers, and the loud failure on CPU
tensors (there is no CPU fallback in the product path)."""
import inspect

import pytest
import torch

from unsamflow_amd import correlation, correlation_native, warp_utils


def test_correlation_signature_matches_reference_plugin():
    sig = inspect.signature(correlation.Correlation.__init__)
    params = list(sig.parameters.values())[1:]
    assert [(p.name, p.default) for p in params] == [
        ("pad_size", 0), ("kernel_size", 0), ("max_displacement", 0),
        ("stride1", 1), ("stride2", 2), ("corr_multiply", 1),
    ]
    fsig = inspect.signature(correlation.CorrelationFunction.forward)
    assert [(p.name, p.default) for p in list(fsig.parameters.values())[3:]] == [
        ("pad_size", 3), ("kernel_size", 3), ("max_displacement", 20),
        ("stride1", 1), ("stride2", 2), ("corr_multiply", 1),
    ]


def test_native_signature_and_attributes():
    m = correlation_native.Correlation(max_displacement=4, kernel_size=1, stride1=1, stride2=1, corr_multiply=1)
    assert m.max_displacement == 4 and m.output_dim == 9 and m.pad_size == 4
    m2 = correlation_native.Correlation(3, "ignored", foo=1)
    assert m2.output_dim == 7


def test_modules_have_no_state():
    m = correlation.Correlation(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=1)
    assert list(m.parameters()) == [] and list(m.buffers()) == [] and m.state_dict() == {}
    assert correlation_native.Correlation().state_dict() == {}


@pytest.mark.parametrize(
    "kw",
    [
        dict(pad_size=4, kernel_size=3, max_displacement=4, stride1=1, stride2=1, corr_multiply=1),
        dict(pad_size=4, kernel_size=1, max_displacement=4, stride1=2, stride2=1, corr_multiply=1),
        dict(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=2, corr_multiply=1),
        dict(pad_size=3, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=1),
        dict(pad_size=5, kernel_size=1, max_displacement=5, stride1=1, stride2=1, corr_multiply=1),
        dict(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=2),
        dict(),  # the Module defaults (kernel_size=0) are not a valid configuration
    ],
)
def test_unsupported_configurations_raise(kw):
    m = correlation.Correlation(**kw)
    x = torch.zeros(1, 2, 3, 3)
    with pytest.raises(NotImplementedError):
        m(x, x)


def test_cpu_tensors_fail_loudly():
    m = correlation.Correlation(pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1, corr_multiply=1)
    x = torch.zeros(1, 2, 3, 3)
    with pytest.raises(RuntimeError, match="no CPU path"):
        m(x, x)
    with pytest.raises(RuntimeError, match="no CPU path"):
        warp_utils.flow_warp(torch.zeros(1, 3, 4, 4), torch.zeros(1, 2, 4, 4))


def test_flow_warp_rejects_other_modes():
    with pytest.raises(NotImplementedError):
        warp_utils.flow_warp(torch.zeros(1, 3, 4, 4), torch.zeros(1, 2, 4, 4), mode="nearest")


def test_mesh_and_norm_grid_semantics():
    g = warp_utils.mesh_grid(2, 3, 4)
    assert g.shape == (2, 2, 3, 4) and g.dtype == torch.int64
    assert g[1, 0, 2, 3] == 3 and g[1, 1, 2, 3] == 2
    n = warp_utils.norm_grid(g.float())
    assert n.shape == (2, 3, 4, 2)
    assert n[0, 0, 0].tolist() == [-1.0, -1.0] and n[0, 2, 3].tolist() == [1.0, 1.0]


def test_occlusion_entry_points_have_no_cpu_path():
    """get_occu_mask_backward / get_corresponding_map run the HIP splat kernel only."""
    with pytest.raises(RuntimeError, match="no CPU path"):
        warp_utils.get_occu_mask_backward(torch.zeros(1, 2, 5, 6))
    with pytest.raises(RuntimeError, match="no CPU path"):
        warp_utils.get_corresponding_map(torch.zeros(1, 2, 5, 6))

