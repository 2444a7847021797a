#!/bin/bash
# correlation forward: edge tiles dispatched last (default) vs XCD-contiguous order; parity, then warm/cold sweep
set -o pipefail
mkdir -p gpurun_out/fe
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_corr_cat.py -k "corr" > gpurun_out/fe/tests.log 2>&1 || { tail -40 gpurun_out/fe/tests.log; exit 1; }
tail -2 gpurun_out/fe/tests.log
timeout -k 10 500 python -u tools/fwdsweep.py --out gpurun_out/fe/edge.json > gpurun_out/fe/edge.log 2>&1 || { tail -20 gpurun_out/fe/edge.log; exit 1; }
USF_LIB=unsamflow_amd/lib/ab/lib_noedge.so timeout -k 10 500 python -u tools/fwdsweep.py --out gpurun_out/fe/noedge.json > gpurun_out/fe/noedge.log 2>&1 || { tail -20 gpurun_out/fe/noedge.log; exit 1; }
echo FEDONE
