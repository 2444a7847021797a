set -o pipefail
export TMPDIR=/tmp KPROF_OPS=corr_bwd KPROF_N=2
R=$(pwd); mkdir -p gpurun_out/abp
for v in o0 o1; do
  export USF_LIB=$R/unsamflow_amd/lib/ab/lib_$v.so
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/abp/${v}_a -o run -- python3 $R/tools/kprof.py > gpurun_out/abp/${v}_a.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/abp/${v}_b -o run -- python3 $R/tools/kprof.py > gpurun_out/abp/${v}_b.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/abp/${v}_c -o run -- python3 $R/tools/kprof.py > gpurun_out/abp/${v}_c.log 2>&1 || exit 1
done
echo ABDONE
