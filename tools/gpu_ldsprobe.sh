#!/bin/bash
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/ldsprobe
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace --output-format csv -d "$R/gpurun_out/ldsprobe" -o run -- "$R/tools/probes/lds_probe" > gpurun_out/ldsprobe/log 2>&1 || { tail gpurun_out/ldsprobe/log; exit 1; }
echo ALLDONE
