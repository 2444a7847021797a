#!/bin/bash
# LDS utilisation of the correlation kernels (one rocprofv3 --pmc pass, kernel trace only).
set -o pipefail
export TMPDIR=/tmp KPROF_OPS=${KPROF_OPS:-corr_fwd_leaky,corr_bwd_leaky} KPROF_N=3
R=$(pwd); mkdir -p gpurun_out/lpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/lpmc/p1 -o run -- python3 $R/tools/kprof.py > gpurun_out/lpmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/lpmc/p2 -o run -- python3 $R/tools/kprof.py > gpurun_out/lpmc/p2.log 2>&1 || exit 1
echo LPMCDONE
