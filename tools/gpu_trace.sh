#!/bin/bash
# Phase traces of the correlation kernels (tools/probes/bin/corr_trace, built in-tree
# on the CPU side). Default: SURVEY config 2 and the KITTI levels at batch 16;
# TRACE_ARGS="fwd 8 128 32 104 9;bwd ..." overrides (the 6th field is the variant).
set -o pipefail
mkdir -p gpurun_out/trace
P=tools/probes/bin/corr_trace
ARGS=${TRACE_ARGS:-"fwd 8 128 32 104;bwd 8 128 32 104;fwd 16 32 64 208;bwd 16 32 64 208;fwd 16 96 16 52;bwd 16 96 16 52"}
IFS=';' read -ra LIST <<< "$ARGS"
for args in "${LIST[@]}"; do
  timeout -k 10 60 $P $args >> gpurun_out/trace/trace.log 2>&1 || { echo "trace $args failed"; tail gpurun_out/trace/trace.log; exit 1; }
done
cat gpurun_out/trace/trace.log
echo TRACEDONE
