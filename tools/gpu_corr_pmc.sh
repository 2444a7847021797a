#!/bin/bash
# SQ activity / instruction-mix passes (separate rocprofv3 runs, --kernel-trace
# only) over the correlation kernels at the KITTI sites and SURVEY config 2.
set -o pipefail
export TMPDIR=/tmp KPROF_OPS=${KPROF_OPS:-corr_fwd,corr_bwd} KPROF_N=3
R=$(pwd); mkdir -p gpurun_out/cpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/cpmc/p1 -o run -- python3 $R/tools/kprof.py > gpurun_out/cpmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/cpmc/p2 -o run -- python3 $R/tools/kprof.py > gpurun_out/cpmc/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-trace --output-format csv -d $R/gpurun_out/cpmc/p3 -o run -- python3 $R/tools/kprof.py > gpurun_out/cpmc/p3.log 2>&1 || exit 1
python tools/pmc_report.py gpurun_out/cpmc | grep -i corr
echo CPMCDONE
