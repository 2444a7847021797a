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
