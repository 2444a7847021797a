#!/bin/bash
# PMC passes (each its own rocprofv3 run; counters only with --kernel-trace).
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
ls -R gpurun_out/pmc | head -30
echo ALLDONE
