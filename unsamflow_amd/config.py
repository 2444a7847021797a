"""Experiment configuration for the benchmark harness.

Only the keys the hot path's callers read are kept (model + loss + the
optimiser/step keys of the train section); values are those of the
reference's JSON configs:

* ``kitti_base()``  — configs/kitti_base.json:27-43 (loss, model), :46-70 (train)
* ``sintel_base()`` — configs/sintel_base.json (same loss/model/train keys)
* ``sintel_mf()``   — configs/sintel_aug+hg+mf.json:3-6 on top of sintel_base
  (mask-feature correlation branch, ``aggregation_type="concat"``)

``load_json`` reads a reference-format JSON file with the one-level
``base_configs`` inheritance + recursive merge of utils/config_parser.py:11-33.
"""
from __future__ import annotations

import copy
import json
import os


class AttrDict(dict):
    """dict with attribute access (the reference uses EasyDict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    @classmethod
    def wrap(cls, obj):
        if isinstance(obj, dict):
            return cls({k: cls.wrap(v) for k, v in obj.items()})
        if isinstance(obj, list):
            return [cls.wrap(v) for v in obj]
        return obj


def merge(base: dict, new: dict) -> dict:
    """Recursive override of ``base`` by ``new`` (config_parser.update_config)."""
    for k, v in new.items():
        if k in base and isinstance(base[k], dict) and isinstance(v, dict):
            merge(base[k], v)
        else:
            base[k] = v
    return base


def load_json(path: str) -> AttrDict:
    with open(path) as f:
        cfg = json.load(f)
    if "base_configs" in cfg:
        with open(os.path.join(os.path.dirname(path), cfg["base_configs"])) as f:
            base = json.load(f)
        cfg = merge(base, cfg)
    return AttrDict.wrap(cfg)


_LOSS = {
    "edge_aware_alpha": 10,
    "occ_from_back": True,
    "smooth_type": "2nd",
    "smooth_edge": "image",
    "type": "unflow",
    "w_l1": 0.15,
    "w_ph_scales": [1.0, 1.0, 1.0, 1.0, 0.0],
    "w_sm": 0,
    "w_ssim": 0.85,
    "w_ternary": 0.0,
    "warp_pad": "border",
    "with_bk": True,
}
_MODEL = {"learned_upsampler": True, "reduce_dense": True, "type": "pwclite"}
_TRAIN = {
    "batch_size": 8,
    "beta": 0.999,
    "bias_decay": 0,
    "lr": 0.0002,
    "max_grad_norm": 10,
    "momentum": 0.9,
    "optim": "adam",
    "weight_decay": 1e-06,
    "lr_scheduler": {
        "module": "OneCycleLR",
        "params": {"max_lr": 0.0004, "pct_start": 0.05, "cycle_momentum": False, "anneal_strategy": "linear"},
    },
    "epoch_num": 200,
    "epoch_size": 1000,
}


def kitti_base() -> AttrDict:
    return AttrDict.wrap({
        "data": {"train_shape": [256, 832], "test_shape": [256, 832]},
        "loss": copy.deepcopy(_LOSS),
        "model": copy.deepcopy(_MODEL),
        "seed": 42,
        "train": copy.deepcopy(_TRAIN),
    })


def sintel_base() -> AttrDict:
    cfg = kitti_base()
    cfg.data = AttrDict.wrap({"test_shape": [448, 1024]})
    return cfg


def sintel_mf() -> AttrDict:
    cfg = sintel_base()
    cfg.model.add_mask_corr = True
    cfg.model.aggregation_type = "concat"
    return cfg
