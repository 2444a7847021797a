"""Golden vectors for the PWCLite + unFlowLoss harness, captured from the
REFERENCE (models/pwclite.py, losses/flow_loss.py) in the build container.

Recipe: stub the un-importable ``correlation_cuda`` and ``cv2``
modules (neither is called here), swap ``models.pwclite.Correlation`` for
``models.correlation_native.Correlation``, pass configs as an attribute dict.
Weights: ``oracle.hashrng.hash_init_`` keyed by parameter name (so this
repo's PWCLite, whose state_dict keys match, gets identical weights without
storing them). Inputs: counter-hash images at 64x128 (KITTI cfg) / 128x256 (mask-feature
cfg, whose level-0 warp divides by H0-1) with B=1, and for the
mask-feature case piecewise-constant segment maps.

Stored: flows_12/flows_21 (all 5 levels), loss / l_ph, per-parameter
gradient sum and abs-sum, and the parameter count.
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))

from oracle import hashrng  # noqa: E402
from unsamflow_amd.config import AttrDict, kitti_base, sintel_mf  # noqa: E402

SIZES = {"kitti": (64, 128), "sintel_mf": (128, 256)}  # mf warps at level 0: needs H0 > 1


def segs(B, seed, H, W, K=4):
    """Piecewise-constant labels in [0,K): 16x16 blocks with hashed ids (float)."""
    bh, bw = H // 16, W // 16
    ids = np.floor(hashrng.uniform((B, 1, bh, bw), seed) * K).astype(np.float32)
    return np.kron(ids, np.ones((1, 1, 16, 16), np.float32))


def run_case(name, cfg, pwclite_mod, flow_loss_mod, corr_native, with_seg):
    H, W = SIZES[name]
    torch.manual_seed(0)
    model = pwclite_mod.PWCLite(AttrDict.wrap(dict(cfg.model)))
    hashrng.hash_init_(model, seed=1)
    loss_fn = flow_loss_mod.unFlowLoss(AttrDict.wrap(dict(cfg.loss)))
    img1 = torch.from_numpy(hashrng.uniform((1, 3, H, W), 11))
    img2 = torch.from_numpy(hashrng.uniform((1, 3, H, W), 12))
    kw = {}
    if with_seg:
        kw = dict(full_seg1=torch.from_numpy(segs(1, 21, H, W)), full_seg2=torch.from_numpy(segs(1, 22, H, W)))
    res = model(img1, img2, with_bk=True, **kw)
    flows = [torch.cat([a, b], 1) for a, b in zip(res["flows_12"], res["flows_21"])]
    loss, l_ph, l_sm, fmean, v1, v2 = loss_fn(flows, img1, img2)
    loss = loss.mean()
    loss.backward()
    out = {
        "loss": np.float64(loss.item()),
        "l_ph": np.float64(l_ph.item()),
        "flow_mean": np.float64(fmean.item()),
        "vis1_sum": np.float64(v1.sum().item()),
        "n_params": np.int64(sum(p.numel() for p in model.parameters())),
        "img1": img1.numpy(),
        "img2": img2.numpy(),
    }
    if with_seg:
        out["seg1"] = kw["full_seg1"].numpy()
        out["seg2"] = kw["full_seg2"].numpy()
    for i, (a, b) in enumerate(zip(res["flows_12"], res["flows_21"])):
        out[f"flow12_{i}"] = a.detach().numpy()
        out[f"flow21_{i}"] = b.detach().numpy()
    names = []
    for n, p in model.named_parameters():
        names.append(n)
        out["gsum:" + n] = np.float64(p.grad.double().sum().item())
        out["gabs:" + n] = np.float64(p.grad.double().abs().sum().item())
    out["param_names"] = np.array(names)
    np.savez_compressed(HERE / f"pwclite_{name}.npz", **out)
    print("pwclite", name, float(loss.detach()), out["n_params"])


def gen_pwclite(ref: Path, here: Path):
    if str(ref) not in sys.path:
        sys.path.insert(0, str(ref))
    sys.modules.setdefault("correlation_cuda", types.ModuleType("correlation_cuda"))
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    from losses import flow_loss as flow_loss_mod
    from models import correlation_native
    from models import pwclite as pwclite_mod

    pwclite_mod.Correlation = correlation_native.Correlation
    run_case("kitti", kitti_base(), pwclite_mod, flow_loss_mod, correlation_native, with_seg=False)
    run_case("sintel_mf", sintel_mf(), pwclite_mod, flow_loss_mod, correlation_native, with_seg=True)


if __name__ == "__main__":
    sys.dont_write_bytecode = True
    gen_pwclite(Path("/root/reference"), HERE)
