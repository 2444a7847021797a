#!/bin/bash
# Per-kernel split of the warp backward on one flow field (WFLOW) at L4 and L3.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out/wprof3
F=${WFLOW:-shift}
for s in "16 32 64 208" "16 64 32 104"; do
  n=$F.$(echo $s | tr ' ' x)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/wprof3/$n" -o run -- python3 "$R/tools/warp_kprof2.py" $F $s > gpurun_out/wprof3/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/wprof3/$n.log; exit 1; }
  echo "== $n"
  python - gpurun_out/wprof3/$n/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'usf' in r['Name'] or 'fillBuffer' in r['Name']:
        print(f"{r['Name'][:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.2f}")
PY
done
echo ALLDONE
