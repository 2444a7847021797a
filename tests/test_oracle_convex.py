"""Pin the convex-upsampler oracle (oracle/upsample.py, restating
UpFlowNetwork at models/pwclite.py:140-166) on the CPU.

The reference's own outputs for this op are the learned-upsampler flows in
tests/golden/pwclite_kitti.npz (kitti_base sets learned_upsampler = true, so
all five returned flows of both directions come out of UpFlowNetwork). The
first test captures the upsampler's inputs inside that golden run and checks
that the oracle reproduces the reference's flows from them; the second checks
the oracle's backward against autograd of its forward (float64)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.hashrng import hash_init_, normal, symmetric
from oracle.torch_ref import OracleCorrelation, oracle_flow_warp
from oracle.upsample import convex_upsample_backward_np, convex_upsample_np
from unsamflow_amd.config import AttrDict, kitti_base
from unsamflow_amd.pwclite import PWCLite, UpFlowNetwork


@pytest.mark.parametrize("batched", [False, True])
def test_convex_oracle_reproduces_reference_flows(batched):
    z = load_golden("pwclite_kitti.npz")
    cfg = kitti_base()
    assert cfg.model.learned_upsampler
    model = PWCLite(AttrDict.wrap(dict(cfg.model)), corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp)
    hash_init_(model, seed=1)
    model.batch_directions = batched
    up = model.output_flow_upsampler
    calls = []
    up.register_forward_hook(lambda m, inp, out: calls.append((inp[0].detach(), inp[1].detach())))
    with torch.no_grad():
        model(torch.from_numpy(z["img1"]), torch.from_numpy(z["img2"]), with_bk=True)
    # 5 levels x 2 directions, or 5 levels with both directions stacked on the batch
    assert len(calls) == (5 if batched else 10)
    B = z["img1"].shape[0]
    for j, (flow, feat) in enumerate(calls):
        with torch.no_grad():
            mask = up.convs(feat).numpy()
        got = convex_upsample_np(flow.numpy(), mask, 4, 0.25)
        lvl = 4 - j % 5  # the decoder returns flows[::-1]
        if batched:
            pairs = [(got[:B], f"flow12_{lvl}"), (got[B:], f"flow21_{lvl}")]
        else:
            pairs = [(got, f"flow{'12' if j < 5 else '21'}_{lvl}")]
        for arr, key in pairs:
            np.testing.assert_allclose(arr, z[key], atol=1e-5, rtol=1e-4, err_msg=key)


def test_convex_oracle_backward_is_the_gradient():
    for f, (B, H, W) in ((4, (2, 5, 7)), (4, (1, 1, 1)), (2, (1, 4, 6)), (8, (1, 3, 2))):
        flow = symmetric((B, 2, H, W), 31 + f, 10.0).astype(np.float64)
        mask = normal((B, 9 * f * f, H, W), 32 + f).astype(np.float64) * 3
        gout = normal((B, 2, f * H, f * W), 33 + f).astype(np.float64)
        tf = torch.from_numpy(flow).requires_grad_(True)
        tm = torch.from_numpy(mask).requires_grad_(True)
        net = UpFlowNetwork(8, f)
        out = net.upsample_flow(tf, 0.25 * tm)  # the model's torch form of pwclite.py:148-160
        out.backward(torch.from_numpy(gout))
        np.testing.assert_allclose(convex_upsample_np(flow, mask, f, 0.25), out.detach().numpy(), atol=1e-9)
        gf, gm = convex_upsample_backward_np(flow, mask, gout, f, 0.25)
        np.testing.assert_allclose(gf, tf.grad.numpy(), atol=1e-9)
        np.testing.assert_allclose(gm, tm.grad.numpy(), atol=1e-9)
