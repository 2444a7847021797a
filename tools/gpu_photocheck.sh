#!/bin/bash
# Photometric + warp GPU tests, then per-kernel device times of the photometric sites.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out/pc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_photometric.py -q -x -m gpu -k "warp or occ or photo" --timeout 120 --timeout-method thread > gpurun_out/pt_photo.log 2>&1 || { tail -30 gpurun_out/pt_photo.log; exit 1; }
tail -1 gpurun_out/pt_photo.log
KPROF_OPS=photo_pair_grad,photo_fwd_grad KPROF_N=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc/kt -o run -- python3 $R/tools/kprof.py > gpurun_out/pc/kt.log 2>&1 || { tail gpurun_out/pc/kt.log; exit 1; }
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/pc/kt/run_kernel_stats.csv')):
    if 'photo' in r['Name']: print(f"{r['Name'][:70]:70s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.2f} min_us={float(r['MinNs'])/1000:.2f} max_us={float(r['MaxNs'])/1000:.2f}")
PY
echo ALLDONE
