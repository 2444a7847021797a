#!/bin/bash
# tile warp backward (branch-free staging, ordered outlier lists, run-merged scatter): tests, timing, profile; FMA-rate probe with DPP.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/bin/fma_rate > gpurun_out/s4_fma_rate.txt 2>&1 || { cat gpurun_out/s4_fma_rate.txt; exit 1; }
cat gpurun_out/s4_fma_rate.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "warp and (tile or scatter_variants)" > gpurun_out/s4_warp_tests.log 2>&1 || { tail -40 gpurun_out/s4_warp_tests.log; exit 1; }
tail -2 gpurun_out/s4_warp_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s4_wprof -o run -- python3 tools/warpab.py --variants 6,8 --out gpurun_out/s4_warpab.json > gpurun_out/s4_wprof.log 2>&1 || { tail -20 gpurun_out/s4_wprof.log; exit 1; }
echo S4DONE
timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --out gpurun_out/s4_corrab_base.json > gpurun_out/s4_corrab_base.log 2>&1 || { tail -20 gpurun_out/s4_corrab_base.log; exit 1; }
USF_LIB=unsamflow_amd/lib/ab/lib_seqdir.so timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --out gpurun_out/s4_corrab_seqdir.json > gpurun_out/s4_corrab_seqdir.log 2>&1 || { tail -20 gpurun_out/s4_corrab_seqdir.log; exit 1; }
grep -h '"op"' gpurun_out/s4_corrab_base.log gpurun_out/s4_corrab_seqdir.log
echo S4BDONE
