"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's hot path.

This package is the parity oracle for the HIP kernels in ``unsamflow_amd``.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker / the timed CPU
baseline — never as a product code path (``unsamflow_amd`` has no CPU
fallback and never imports this package).

Contents
--------
* :mod:`oracle.corr` — correlation forward/backward restating
  ``models/correlation_native.py:13-23`` (the north star's named oracle) and
  the CUDA plugin's backward formulas (``correlation_cuda_kernel.cu:116-300``).
* :mod:`oracle.warp` — ``flow_warp`` (``utils/warp_utils.py:97-106``) with the
  ATen ``grid_sampler_2d`` CPU bilinear algorithm (torch 2.10,
  aten/src/ATen/native/cpu/GridSamplerKernel.cpp — third-party, not in
  /root/reference) restated in float32 numpy.
* :mod:`oracle.hashrng` — counter-hash generator for bit-reproducible inputs.
* :mod:`oracle.torch_ref` — torch-CPU modules with reference semantics used to
  drive the PWCLite harness on CPU (gloo tests, CPU baseline).

Pinning: every function here is checked against golden vectors captured by
importing the reference itself in the survey container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.
"""
