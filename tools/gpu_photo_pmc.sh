#!/bin/bash
# PMC passes (occupancy/activity, instruction mix) over the photometric pair kernels, per variant.
set -o pipefail
export TMPDIR=/tmp KPROF_OPS=photo_pair_grad KPROF_N=3
R=$(pwd); mkdir -p gpurun_out/ppv
for v in ${PHOTO_VARIANTS:-0 2}; do
  export USF_PHOTO_VARIANT=$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/ppv/v$v/p1 -o run -- python3 $R/tools/kprof.py > gpurun_out/ppv/v$v.p1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/ppv/v$v/p2 -o run -- python3 $R/tools/kprof.py > gpurun_out/ppv/v$v.p2.log 2>&1 || exit 1
  echo "== variant $v"; python tools/pmc_report.py gpurun_out/ppv/v$v | grep -i photo
done
