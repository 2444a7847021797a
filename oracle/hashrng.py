"""TEST INFRASTRUCTURE ONLY — counter-hash random numbers (see oracle/__init__.py).

``uniform(shape, seed)`` and ``normal(shape, seed)`` are pure functions of
(shape, seed, element index): splitmix64 of ``seed * 2^32 + index`` mapped to
[0, 1) with 24 bits, so the same values come out on every machine and numpy
version (no reliance on torch/numpy RNG stream stability). Used to build large
test inputs whose expected reductions are recorded in tests/golden, and to
initialise PWCLite deterministically by parameter name.
"""
from __future__ import annotations

import zlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def _splitmix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(shape, seed: int) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    idx = np.arange(n, dtype=np.uint64) + (np.uint64(seed & 0xFFFFFFFF) << np.uint64(32))
    bits = _splitmix(idx) >> np.uint64(40)  # top 24 bits
    return (bits.astype(np.float64) / float(1 << 24)).astype(np.float32).reshape(shape)


def symmetric(shape, seed: int, scale: float = 1.0) -> np.ndarray:
    """Uniform in [-scale, scale)."""
    return ((uniform(shape, seed) * np.float32(2) - np.float32(1)) * np.float32(scale)).astype(np.float32)


def normal(shape, seed: int) -> np.ndarray:
    """Approximately N(0,1) (Box-Muller on two hash streams)."""
    u1 = uniform(shape, seed).astype(np.float64)
    u2 = uniform(shape, seed ^ 0x5BD1E995).astype(np.float64)
    r = np.sqrt(-2.0 * np.log1p(-u1))  # 1-u1 in (0, 1]
    return (r * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def name_seed(name: str, seed: int = 0) -> int:
    """Stable 32-bit seed from a parameter name."""
    return (zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF


def hash_init_(module, seed: int = 0) -> None:
    """Deterministically overwrite every parameter of ``module`` (in place).

    weights ~ U[-1/sqrt(fan_in), 1/sqrt(fan_in)) (the scale of PyTorch's
    default Conv2d init), biases likewise; keyed by parameter name so two
    implementations with identical state_dict keys get identical weights.
    """
    import torch

    with torch.no_grad():
        for name, p in module.named_parameters():
            fan_in = int(np.prod(p.shape[1:])) if p.dim() > 1 else max(1, p.shape[0])
            if name.endswith("bias"):
                # bias bound uses the owning weight's fan-in when available
                wname = name[: -len("bias")] + "weight"
                w = dict(module.named_parameters()).get(wname)
                if w is not None and w.dim() > 1:
                    fan_in = int(np.prod(w.shape[1:]))
            bound = 1.0 / np.sqrt(fan_in)
            v = symmetric(tuple(p.shape), name_seed(name, seed), bound)
            p.copy_(torch.from_numpy(v))
