#!/bin/bash
# Current-tree measurements of the other configurations: the Sintel mask-feature step
# (SURVEY config 5 per GPU) and graph replay of the KITTI step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --config sintel_mf --no-cpu-baseline > gpurun_out/bench_sintel_mf.json 2> gpurun_out/bench_sintel_mf.err || { echo "sintel failed"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench_sintel_mf.err | tail -20; exit 1; }
head -c 400 gpurun_out/bench_sintel_mf.json; echo
timeout -k 10 600 python bench.py --graph --no-cpu-baseline > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || { echo "graph failed"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench_graph.err | tail -20; exit 1; }
head -c 400 gpurun_out/bench_graph.json; echo
echo ALLDONE
