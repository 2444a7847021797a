#!/bin/bash
# PMC passes over tools/kprof.py (each its own rocprofv3 run; counters only with
# --kernel-trace, never with sys/runtime/hip traces). PASSES selects passes:
# 1 = wave occupancy/activity, 2 = instruction mix + LDS conflicts,
# 3 = FETCH_SIZE, 4 = WRITE_SIZE (3+4 feed tools/pmc_traffic.py).
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
SETS=("" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE")
for i in ${PASSES:-1 2 3 4}; do
  timeout -k 10 300 rocprofv3 --pmc ${SETS[$i]} --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
ls -R gpurun_out/pmc | head -30
echo ALLDONE
