"""PWCLite + unFlowLoss with the HIP hot path on the GPU against the
REFERENCE's captured outputs (tests/golden/pwclite_*.npz).

Tolerance: flows atol 1e-4 / rtol 1e-3, loss rtol 1e-4, per-parameter
gradient sums within 2e-3 of the gradient abs-sum — the convolutions run on
MIOpen (GPU) vs oneDNN (CPU) in the capture, so agreement is at fp32
conv-reduction-order level, not bitwise.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.hashrng import hash_init_
from unsamflow_amd.config import AttrDict, kitti_base, sintel_mf

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,cfg_fn", [("kitti", kitti_base), ("sintel_mf", sintel_mf)])
def test_pwclite_hip_matches_reference(hip_device, name, cfg_fn):
    from unsamflow_amd.flow_loss import unFlowLoss
    from unsamflow_amd.pwclite import PWCLite

    z = load_golden(f"pwclite_{name}.npz")
    cfg = cfg_fn()
    model = PWCLite(AttrDict.wrap(dict(cfg.model))).to(hip_device)
    hash_init_(model, seed=1)
    loss_fn = unFlowLoss(AttrDict.wrap(dict(cfg.loss)))
    img1 = torch.from_numpy(z["img1"]).to(hip_device)
    img2 = torch.from_numpy(z["img2"]).to(hip_device)
    kw = {}
    if "seg1" in z:
        kw = dict(full_seg1=torch.from_numpy(z["seg1"]).to(hip_device),
                  full_seg2=torch.from_numpy(z["seg2"]).to(hip_device))
    res = model(img1, img2, with_bk=True, **kw)
    flows = [torch.cat([a, b], 1) for a, b in zip(res["flows_12"], res["flows_21"])]
    loss, l_ph, _, _, _, _ = loss_fn(flows, img1, img2)
    loss = loss.mean()
    loss.backward()
    for i in range(5):
        np.testing.assert_allclose(res["flows_12"][i].detach().cpu().numpy(), z[f"flow12_{i}"], atol=1e-4, rtol=1e-3)
        np.testing.assert_allclose(res["flows_21"][i].detach().cpu().numpy(), z[f"flow21_{i}"], atol=1e-4, rtol=1e-3)
    assert abs(loss.item() - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    for n, p in model.named_parameters():
        gs, ga = float(z["gsum:" + n]), float(z["gabs:" + n])
        assert abs(p.grad.double().sum().item() - gs) <= 2e-3 * ga + 1e-8, n
        assert abs(p.grad.double().abs().sum().item() - ga) <= 2e-3 * ga + 1e-8, n


def test_smoke_step(hip_device):
    from __graft_entry__ import smoke_step

    smoke_step(hip_device)


def test_train_step_full_kitti_size(hip_device):
    """One real-size step (B=2, 832x256) runs and updates the weights."""
    from unsamflow_amd.harness import TrainStep, synthetic_pair

    step = TrainStep(kitti_base(), hip_device)
    img1, img2, _, _ = synthetic_pair(2, 256, 832, hip_device)
    w0 = step.module.conv_1x1[4][0].weight.detach().clone()
    loss = step(img1, img2)
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    assert not torch.equal(w0, step.module.conv_1x1[4][0].weight)


def test_graphed_step_matches_eager_steps(hip_device):
    """harness.GraphedTrainStep (the step captured into a HIP graph and replayed)
    trains like TrainStep: same losses and parameters after the same number of
    steps from the same state (up to the warp backward's atomic summation order)."""
    from oracle.hashrng import uniform
    from unsamflow_amd.config import kitti_base
    from unsamflow_amd.harness import GraphedTrainStep, TrainStep

    im1 = torch.from_numpy(uniform((2, 3, 64, 128), 31)).to(hip_device)
    im2 = torch.from_numpy(uniform((2, 3, 64, 128), 32)).to(hip_device)
    eager = TrainStep(kitti_base(), hip_device, capturable=True)
    graphed = TrainStep(kitti_base(), hip_device, capturable=True)
    losses_e = [float(eager(im1, im2)) for _ in range(3)]
    g = GraphedTrainStep(graphed, im1, im2, warmup=1)  # 1 eager warm-up step, then capture
    losses_g = [float(g()) for _ in range(2)]
    torch.cuda.synchronize()
    # the graph's first replay is step 2 (the warm-up was step 1)
    np.testing.assert_allclose(losses_g, losses_e[1:], rtol=1e-4)
    for (n, pe), pg in zip(eager.module.named_parameters(), graphed.module.parameters()):
        torch.testing.assert_close(pg, pe, atol=1e-5, rtol=1e-4, msg=n)
    assert float(graphed.optimizer.param_groups[0]["lr"]) == pytest.approx(
        float(eager.optimizer.param_groups[0]["lr"]))
