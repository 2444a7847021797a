#!/bin/bash
# Warp parity tests, then the per-kernel split of the warp backward (tools/gpu_wprof2.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_photometric.py -q -x -m gpu -k "warp or occ or photo" --timeout 120 --timeout-method thread > gpurun_out/pt_warp.log 2>&1 || { tail -30 gpurun_out/pt_warp.log; exit 1; }
tail -2 gpurun_out/pt_warp.log
bash tools/gpu_wprof2.sh > gpurun_out/wprof2.log 2>&1 || { tail gpurun_out/wprof2.log; exit 1; }
for d in gpurun_out/wprof2/*/; do echo "== $d"; python - "$d" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1]+'run_kernel_stats.csv')):
    if 'usf' in r['Name'] or 'fillBuffer' in r['Name']:
        print(f"{r['Name'][:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.2f}")
PY
done
echo ALLDONE
