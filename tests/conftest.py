"""pytest configuration: the ``gpu`` marker and shared helpers.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors, host logic,
C-ABI load/export checks, CPU harness tests (oracle-backed ops injected).
``-m gpu`` runs on an MI355X: HIP kernels vs the oracle / golden vectors.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and the built HIP library")


def load_golden(name: str):
    return dict(np.load(GOLDEN / name, allow_pickle=False))


def golden_files(prefix: str):
    return sorted(p.name for p in GOLDEN.glob(f"{prefix}*.npz"))


@pytest.fixture(scope="session")
def hip_device():
    """cuda:0 with the HIP library loaded; fails (not skips) if the library is missing on a GPU box."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device visible")
    from unsamflow_amd import _lib

    _lib.load()  # raises if missing: GPU tests must run the native path
    return torch.device("cuda:0")
