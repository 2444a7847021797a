#!/bin/bash
# GPU-box script: phase timing of the correlation kernels at the KITTI level
# shapes (tools/probes/corr_trace, prebuilt here by hipcc).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/corr_trace.txt; : > $out
for args in "fwd 8 192 4 13" "fwd 8 128 8 26" "fwd 8 96 16 52" "fwd 8 64 32 104" "fwd 8 32 64 208" \
            "bwd 8 192 4 13" "bwd 8 128 8 26" "bwd 8 96 16 52" "bwd 8 64 32 104" "bwd 8 32 64 208" ${EXTRA_TRACE}; do
  timeout -k 5 60 ./tools/probes/corr_trace $args >> $out 2>&1 || { echo "trace failed: $args"; cat $out; exit 1; }
done
cat $out
