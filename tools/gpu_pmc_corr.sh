#!/bin/bash
# PMC wave-state passes over the correlation sites only (tools/kprof.py with
# KPROF_OPS), each pass its own rocprofv3 run, --kernel-trace only.
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
export KPROF_OPS=${KPROF_OPS:-corr_fwd,corr_bwd,corr_bwd_leaky,warp_bwd} KPROF_N=${KPROF_N:-3}
SETS=("" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum")
for i in ${PASSES:-1 2 3 4}; do
  timeout -s KILL 120 rocprofv3 --pmc ${SETS[$i]} --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 tools/pmc_report.py gpurun_out/pmc > gpurun_out/pmc/report.txt && cat gpurun_out/pmc/report.txt
echo ALLDONE
