#!/bin/bash
# warp corner-pair loads: parity (warp goldens, oracle, graph replay), then device time with and without
set -o pipefail
mkdir -p gpurun_out/wp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_graph_replay.py tests/test_gpu_occ_bidirection.py -k "warp or harness or graph or occ" > gpurun_out/wp/tests.log 2>&1 || { tail -40 gpurun_out/wp/tests.log; exit 1; }
tail -2 gpurun_out/wp/tests.log
timeout -k 10 300 python -u tools/sitebench.py --ops warp_fwd,warp_bwd --out gpurun_out/wp/pair.json > gpurun_out/wp/pair.log 2>&1 || { tail -20 gpurun_out/wp/pair.log; exit 1; }
USF_LIB=unsamflow_amd/lib/ab/lib_nopair.so timeout -k 10 300 python -u tools/sitebench.py --ops warp_fwd,warp_bwd --out gpurun_out/wp/nopair.json > gpurun_out/wp/nopair.log 2>&1 || { tail -20 gpurun_out/wp/nopair.log; exit 1; }
echo WPDONE
