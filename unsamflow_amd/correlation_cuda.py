"""``correlation_cuda``-compatible module: the reference plugin's Python-visible
ABI (pybind ``forward``/``backward``, models/correlation_package/
correlation_cuda.cc:167-170) implemented on libunsamflow_hip.so.

With ``sys.modules["correlation_cuda"] = unsamflow_amd.correlation_cuda`` the
reference's own ``models/correlation_package/correlation.py`` runs unmodified
on MI355X. Semantics of the reference glue are kept:

* ``forward(input1, input2, rInput1, rInput2, output, pad_size, kernel_size,
  max_displacement, stride1, stride2, corr_multiply) -> int`` resizes ``output``
  to [B, (2d+1)^2, H, W] and fills it (correlation_cuda.cc:10-86);
* ``backward(input1, input2, rInput1, rInput2, gradOutput, gradInput1,
  gradInput2, pad_size, ...) -> int`` resizes the two gradient tensors to the
  input shape and fills them (:88-165);
* return 1 on success; a failed launch raises ``RuntimeError`` (the reference
  raises ``AT_ERROR("CUDA call failed")``, :80-82 / :160-162).

The padded NHWC scratch tensors ``rInput1/2`` of the CUDA design are not
needed (the HIP kernels stage their halos in LDS); they are left empty.
Unsupported argument combinations raise ``NotImplementedError`` (see
unsamflow_amd.correlation.check_supported).
"""
from __future__ import annotations

import torch

from . import ops
from .correlation import check_supported


def forward(input1, input2, rInput1, rInput2, output, pad_size, kernel_size, max_displacement,
            stride1, stride2, corr_multiply) -> int:
    d = check_supported(pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply)
    B, _, H, W = input1.shape
    K = 2 * d + 1
    output.resize_(B, K * K, H, W)
    ops.corr_forward(input1, input2, d, out=output)
    return 1


def backward(input1, input2, rInput1, rInput2, gradOutput, gradInput1, gradInput2, pad_size,
             kernel_size, max_displacement, stride1, stride2, corr_multiply) -> int:
    d = check_supported(pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply)
    gradInput1.resize_(input1.shape)
    gradInput2.resize_(input2.shape)
    ops.corr_backward(input1, input2, gradOutput, d, True, True, gx1_out=gradInput1, gx2_out=gradInput2)
    return 1


__all__ = ["forward", "backward"]
_ = torch  # re-exported tensor type used in the signatures above
