#!/bin/bash
# Phase traces of the correlation kernels (tools/probes/corr_trace, built in-tree
# on the CPU side): SURVEY config 2 and the small KITTI levels at batch 16.
set -o pipefail
mkdir -p gpurun_out/trace
P=tools/probes/corr_trace
for args in "fwd 8 128 32 104" "bwd 8 128 32 104" "fwd 16 192 4 13" "bwd 16 192 4 13" \
            "fwd 16 128 8 26" "bwd 16 128 8 26" "fwd 16 96 16 52" "bwd 16 96 16 52"; do
  timeout -k 10 60 $P $args >> gpurun_out/trace/trace.log 2>&1 || { echo "trace $args failed"; tail gpurun_out/trace/trace.log; exit 1; }
done
cat gpurun_out/trace/trace.log
echo TRACEDONE
