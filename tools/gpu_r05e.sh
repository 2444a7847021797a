#!/bin/bash
# Round-5 pass E (gpurun_out/r05e/): persistent warp v3 -- tests and timing; corr backward
# order A/B: this tree (whole (sample, direction) per XCD chunk on ring grids) vs
# USF_BWD_SAMPLE_RING=0 (lib_sampring0).
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_persist.py tests/test_gpu_graph_replay.py tests/test_gpu_occ_bidirection.py tests/test_gpu_parity.py -k "persist or replay or warp or occ" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/persist_ab.py --out $O/persist_ab.json > $O/persist_ab.log 2>&1 || { tail -20 $O/persist_ab.log; exit 1; }
rm -rf gpurun_out/bab
OP=bwd AB=unsamflow_amd/lib/ab/lib_sampring0.so timeout -k 10 900 bash tools/gpu_corr_ab.sh > $O/ab_sampring0.log 2>&1 || { tail -30 $O/ab_sampring0.log; exit 1; }
tail -1 $O/ab_sampring0.log; cp -r gpurun_out/bab $O/bab_sampring0
echo R05E_DONE
