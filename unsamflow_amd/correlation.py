"""Drop-in for ``models/correlation_package/correlation.py`` (the reference's
native correlation plugin), backed by the gfx950 HIP kernels.

Same public surface as the reference:

* ``CorrelationFunction.apply(input1, input2, pad_size, kernel_size,
  max_displacement, stride1, stride2, corr_multiply)`` (correlation.py:7-72)
* ``Correlation(pad_size=0, kernel_size=0, max_displacement=0, stride1=1,
  stride2=2, corr_multiply=1)`` with ``forward(input1, input2)``
  (correlation.py:75-102), constructed by PWCLite as
  ``Correlation(pad_size=4, kernel_size=1, max_displacement=4, stride1=1,
  stride2=1, corr_multiply=1)`` (pwclite.py:208-215).

Supported subset (everything any reference caller uses): kernel_size=1,
stride1=stride2=1, pad_size == max_displacement in [1, 4], corr_multiply=1,
fp32 tensors on a ROCm device. Anything else raises ``NotImplementedError``.
The output is NOT saved for backward (PWCLite applies LeakyReLU in place on
it, pwclite.py:189,308), and the module registers no parameters or buffers,
so PWCLite's ``state_dict`` keys are unchanged.
"""
from __future__ import annotations

import torch
from torch.autograd import Function
from torch.nn import Module

from . import ops

MAX_SUPPORTED_DISPLACEMENT = 4


def check_supported(pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply) -> int:
    """Validate the plugin arguments; return the displacement radius d."""
    d = int(max_displacement)
    if kernel_size != 1:
        raise NotImplementedError(f"Correlation kernel_size={kernel_size} (only 1 is supported)")
    if stride1 != 1 or stride2 != 1:
        raise NotImplementedError(f"Correlation strides ({stride1}, {stride2}) (only 1, 1 is supported)")
    if pad_size != d:
        raise NotImplementedError(f"Correlation pad_size={pad_size} != max_displacement={d}")
    if corr_multiply != 1:
        raise NotImplementedError(f"Correlation corr_multiply={corr_multiply} (only 1 is supported)")
    if not 1 <= d <= MAX_SUPPORTED_DISPLACEMENT:
        raise NotImplementedError(f"Correlation max_displacement={d} not in [1, {MAX_SUPPORTED_DISPLACEMENT}]")
    return d


class CorrelationFunction(Function):
    """autograd Function with the reference's argument list and defaults."""

    @staticmethod
    def forward(ctx, input1, input2, pad_size=3, kernel_size=3, max_displacement=20,
                stride1=1, stride2=2, corr_multiply=1):
        d = check_supported(pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply)
        ctx.save_for_backward(input1, input2)
        ctx.max_displacement = d
        return ops.corr_forward(input1, input2, d)

    @staticmethod
    def backward(ctx, grad_output):
        input1, input2 = ctx.saved_tensors
        need1, need2 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        g1, g2 = ops.corr_backward(input1, input2, grad_output, ctx.max_displacement, need1, need2)
        return g1, g2, None, None, None, None, None, None


class Correlation(Module):
    def __init__(self, pad_size=0, kernel_size=0, max_displacement=0, stride1=1, stride2=2,
                 corr_multiply=1):
        super().__init__()
        self.pad_size = pad_size
        self.kernel_size = kernel_size
        self.max_displacement = max_displacement
        self.stride1 = stride1
        self.stride2 = stride2
        self.corr_multiply = corr_multiply

    def forward(self, input1: torch.Tensor, input2: torch.Tensor) -> torch.Tensor:
        return CorrelationFunction.apply(
            input1, input2, self.pad_size, self.kernel_size, self.max_displacement,
            self.stride1, self.stride2, self.corr_multiply,
        )

    def extra_repr(self) -> str:
        return (f"pad_size={self.pad_size}, kernel_size={self.kernel_size}, "
                f"max_displacement={self.max_displacement}, stride1={self.stride1}, "
                f"stride2={self.stride2}, corr_multiply={self.corr_multiply}")
