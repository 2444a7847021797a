#!/bin/bash
# Per-kernel split of the warp backward (binned gather) at L4 / L3 / L1, smooth +-2 px field.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out/wprof2
for s in "16 32 64 208" "16 64 32 104" "16 128 8 26"; do
  n=$(echo $s | tr ' ' x)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/wprof2/$n" -o run -- python3 "$R/tools/warp_kprof.py" $s > gpurun_out/wprof2/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/wprof2/$n.log; exit 1; }
  echo "== $n"; cut -d, -f1-4 gpurun_out/wprof2/$n/run_kernel_stats.csv | cut -c1-160
done
echo ALLDONE
