"""The PWCLite + unFlowLoss harness (this repo's rebuild of the hot path's
callers) against the REFERENCE's own outputs (tests/golden/pwclite_*.npz),
on CPU with the oracle ops injected for correlation and warp."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.hashrng import hash_init_
from oracle.torch_ref import OracleCorrelation, oracle_flow_warp, oracle_occu_mask_backward
from unsamflow_amd.config import AttrDict, kitti_base, sintel_mf
from unsamflow_amd.flow_loss import unFlowLoss
from unsamflow_amd.pwclite import PWCLite


def _run(name, cfg):
    z = load_golden(f"pwclite_{name}.npz")
    model = PWCLite(AttrDict.wrap(dict(cfg.model)), corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp)
    hash_init_(model, seed=1)
    loss_fn = unFlowLoss(AttrDict.wrap(dict(cfg.loss)), warp_fn=oracle_flow_warp,
                         occ_backward_fn=oracle_occu_mask_backward)
    img1, img2 = torch.from_numpy(z["img1"]), torch.from_numpy(z["img2"])
    kw = {}
    if "seg1" in z:
        kw = dict(full_seg1=torch.from_numpy(z["seg1"]), full_seg2=torch.from_numpy(z["seg2"]))
    res = model(img1, img2, with_bk=True, **kw)
    flows = [torch.cat([a, b], 1) for a, b in zip(res["flows_12"], res["flows_21"])]
    loss, l_ph, _, fmean, v1, _ = loss_fn(flows, img1, img2)
    loss = loss.mean()
    loss.backward()
    return z, model, res, loss, l_ph, fmean, v1


@pytest.mark.parametrize("name,cfg_fn", [("kitti", kitti_base), ("sintel_mf", sintel_mf)])
def test_pwclite_matches_reference(name, cfg_fn):
    z, model, res, loss, l_ph, fmean, v1 = _run(name, cfg_fn())
    assert sum(p.numel() for p in model.parameters()) == int(z["n_params"])
    assert [n for n, _ in model.named_parameters()] == list(z["param_names"])
    for i in range(5):
        np.testing.assert_allclose(res["flows_12"][i].detach().numpy(), z[f"flow12_{i}"], atol=1e-5, rtol=1e-4)
        np.testing.assert_allclose(res["flows_21"][i].detach().numpy(), z[f"flow21_{i}"], atol=1e-5, rtol=1e-4)
    assert abs(loss.item() - float(z["loss"])) <= 1e-6 * abs(float(z["loss"])) + 1e-7
    assert abs(l_ph.item() - float(z["l_ph"])) <= 1e-6 * abs(float(z["l_ph"])) + 1e-7
    assert abs(fmean.item() - float(z["flow_mean"])) <= 1e-5
    assert v1.sum().item() == float(z["vis1_sum"])
    for n, p in model.named_parameters():
        gs, ga = float(z["gsum:" + n]), float(z["gabs:" + n])
        assert abs(p.grad.double().abs().sum().item() - ga) <= 1e-4 * ga + 1e-9, n
        assert abs(p.grad.double().sum().item() - gs) <= 1e-4 * ga + 1e-9, n


def test_state_dict_keys_are_reference_compatible():
    z = load_golden("pwclite_kitti.npz")
    model = PWCLite(kitti_base().model, corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp)
    assert list(model.state_dict().keys()) == list(z["param_names"])


def test_train_step_runs_on_cpu_with_oracle_ops():
    from unsamflow_amd.harness import TrainStep, synthetic_pair

    cfg = kitti_base()
    step = TrainStep(cfg, "cpu", corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                     occ_backward_fn=oracle_occu_mask_backward)
    img1, img2, _, _ = synthetic_pair(1, 64, 128, "cpu")
    before = [p.detach().clone() for p in step.module.parameters()]
    loss = step(img1, img2)
    assert torch.isfinite(loss)
    changed = sum(int(not torch.equal(a, p)) for a, p in zip(before, step.module.parameters()))
    assert changed > 0.9 * len(before)


def test_homography_smoothness_is_rejected():
    cfg = kitti_base()
    cfg.loss.w_sm = 0.1
    cfg.loss.smooth_type = "homography"
    loss_fn = unFlowLoss(cfg.loss, warp_fn=oracle_flow_warp, occ_backward_fn=oracle_occu_mask_backward)
    flows = [torch.zeros(1, 4, 64 >> i, 128 >> i) for i in range(5)]
    with pytest.raises(NotImplementedError):
        loss_fn(flows, torch.rand(1, 3, 64, 128), torch.rand(1, 3, 64, 128))
