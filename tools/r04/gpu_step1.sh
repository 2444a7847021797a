#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_photometric.py tests/test_gpu_fullsize.py tests/test_capi.py > gpurun_out/step1_tests.log 2>&1 || { tail -30 gpurun_out/step1_tests.log; exit 1; }
tail -3 gpurun_out/step1_tests.log
bash tools/r04/gpu_lds_pmc.sh
