#!/bin/bash
# Round-5 pass D (outputs under gpurun_out/r05d/): the revised persistent warp/occ forms --
# their tests, graph replay, the warp/occlusion parity tests, then persistent vs per-call timing.
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_persist.py tests/test_gpu_graph_replay.py tests/test_gpu_occ_bidirection.py "tests/test_gpu_parity.py" -k "persist or replay or warp or occ" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/persist_ab.py --out $O/persist_ab.json > $O/persist_ab.log 2>&1 || { tail -20 $O/persist_ab.log; exit 1; }
echo R05D_DONE
