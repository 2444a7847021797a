"""Drop-in for ``models/correlation_native.py`` (its constructor form),
computed by the same gfx950 kernels as :mod:`unsamflow_amd.correlation`.

``Correlation(max_displacement=4, *args, **kwargs)`` — extra constructor
arguments are accepted and ignored exactly as in the reference
(correlation_native.py:7), and ``output_dim`` / ``pad_size`` are exposed with
the same meaning (:9-11). ``forward(x1, x2)`` returns [B,(2d+1)^2,H,W].
"""
from __future__ import annotations

import torch
from torch.nn import Module

from .correlation import CorrelationFunction


class Correlation(Module):
    def __init__(self, max_displacement=4, *args, **kwargs):
        super().__init__()
        self.max_displacement = max_displacement
        self.output_dim = 2 * self.max_displacement + 1
        self.pad_size = self.max_displacement

    def forward(self, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
        d = self.max_displacement
        return CorrelationFunction.apply(x1, x2, d, 1, d, 1, 1, 1)
