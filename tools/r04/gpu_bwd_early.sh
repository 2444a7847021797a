#!/bin/bash
# correlation backward with the stage-0 DMA ahead of the g slice (USF_BWD_EARLY): parity, then A/B device time
set -o pipefail
mkdir -p gpurun_out/be
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_corr_cat.py -k "corr" > gpurun_out/be/tests.log 2>&1 || { tail -40 gpurun_out/be/tests.log; exit 1; }
tail -2 gpurun_out/be/tests.log
for i in 1 2; do
timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --out gpurun_out/be/early$i.json > gpurun_out/be/early$i.log 2>&1 || { tail -20 gpurun_out/be/early$i.log; exit 1; }
USF_LIB=unsamflow_amd/lib/ab/lib_noearly.so timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --out gpurun_out/be/base$i.json > gpurun_out/be/base$i.log 2>&1 || { tail -20 gpurun_out/be/base$i.log; exit 1; }
done
echo BEDONE
