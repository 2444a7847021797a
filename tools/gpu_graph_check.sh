#!/bin/bash
# Graph-replay parity of the hot-path calls, the warp/occlusion GPU tests, then ONE
# bounded graphed bench run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_replay.py -x -v --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -3 gpurun_out/graph_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "warp or occ or photo" --timeout 120 --timeout-method thread > gpurun_out/warp_tests.log 2>&1 || { tail -40 gpurun_out/warp_tests.log; exit 1; }
tail -2 gpurun_out/warp_tests.log
USF_ALLOW_GRAPH_BENCH=1 timeout -k 10 240 python -u bench.py --graph --steps 5 --warmup 3 --no-cpu-baseline --no-replay > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || { echo "graph bench rc=$?"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench_graph.err | tail -20; exit 1; }
head -c 300 gpurun_out/bench_graph.json; echo
echo ALLDONE
