#!/bin/bash
# warp tile backward: parity tests first, then timing vs the binned gather; photometric / full-size tests; LDS PMC.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "warp and (tile or scatter_variants or golden or small)" > gpurun_out/s2_warp_tests.log 2>&1 || { tail -40 gpurun_out/s2_warp_tests.log; exit 1; }
tail -3 gpurun_out/s2_warp_tests.log
timeout -k 10 300 python -u tools/warpab.py --variants 6,8,7 --out gpurun_out/s2_warpab.json > gpurun_out/s2_warpab.log 2>&1 || { tail -20 gpurun_out/s2_warpab.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_photometric.py tests/test_gpu_fullsize.py tests/test_gpu_graph_replay.py tests/test_gpu_occ_bidirection.py > gpurun_out/s2_tests.log 2>&1 || { tail -40 gpurun_out/s2_tests.log; exit 1; }
tail -3 gpurun_out/s2_tests.log
bash tools/r04/gpu_lds_pmc.sh
