set -o pipefail
export TMPDIR=/tmp KPROF_OPS=${KPROF_OPS:-photo_pair_grad,photo_bwd} KPROF_N=3
R=$(pwd); mkdir -p gpurun_out/pp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp/kt -o run -- python3 $R/tools/kprof.py > gpurun_out/pp/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pp/p1 -o run -- python3 $R/tools/kprof.py > gpurun_out/pp/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pp/p2 -o run -- python3 $R/tools/kprof.py > gpurun_out/pp/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pp/p3 -o run -- python3 $R/tools/kprof.py > gpurun_out/pp/p3.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pp/p4 -o run -- python3 $R/tools/kprof.py > gpurun_out/pp/p4.log 2>&1 || exit 1
echo PPDONE
