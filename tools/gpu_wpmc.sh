#!/bin/bash
# PMC passes of the warp backward kernels at one decoder site (+-2 px field).
set -o pipefail
export TMPDIR=/tmp KPROF_N=5
R=$(pwd); mkdir -p gpurun_out/wpmc
S=${WSHAPE:-16 32 64 208}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/wpmc/p$i" -o run -- python3 "$R/tools/warp_kprof.py" $S > gpurun_out/wpmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/wpmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, collections
rows=collections.defaultdict(lambda: collections.defaultdict(list))
for p in (1,2,3,4):
    for r in csv.DictReader(open(f'gpurun_out/wpmc/p{p}/run_counter_collection.csv')):
        if 'usf' not in r['Kernel_Name']: continue
        rows[r['Kernel_Name'][:70]][r['Counter_Name']].append(float(r['Counter_Value']))
for k,d in rows.items():
    print(k); print('   ', {c: round(sum(v)/len(v)) for c,v in sorted(d.items())})
PY
echo ALLDONE
