#!/bin/bash
# GPU-box script: small-level correlation parity tests + per-site device times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_corr_cat.py tests/test_gpu_graph_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1
rc=$?; tail -5 gpurun_out/small_tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAIL" gpurun_out/small_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/sitebench.py --ops ${OPS:-corr_fwd_leaky,corr_bwd_leaky} --out gpurun_out/small_sites.json > gpurun_out/small_sites.log 2>&1 || { tail -20 gpurun_out/small_sites.log; exit 1; }
cat gpurun_out/small_sites.log
