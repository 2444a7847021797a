#!/bin/bash
# Correlation GPU parity tests, then the forward/backward timings at the decoder sites and SURVEY configs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_corr_cat.py tests/test_gpu_harness.py -q -x -m gpu -k "corr or harness or pwclite" --timeout 120 --timeout-method thread > gpurun_out/pt_corr.log 2>&1 || { tail -30 gpurun_out/pt_corr.log; exit 1; }
tail -2 gpurun_out/pt_corr.log
timeout -k 10 200 python tools/corrab.py --ops fwd,bwd,leaky --out gpurun_out/corrab.json > gpurun_out/corrab.log 2>&1 || { tail gpurun_out/corrab.log; exit 1; }
cat gpurun_out/corrab.log | grep -v amdgpu.ids
echo ALLDONE
