#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, --kernel-trace only) of
# tools/kprof.py for every A/B build, restricted to KPROF_OPS sites.
set -o pipefail
export TMPDIR=/tmp KPROF_OPS=${KPROF_OPS:-corr_bwd_leaky} KPROF_N=${KPROF_N:-3}
R=$(pwd); mkdir -p gpurun_out/abpmc
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    USF_LIB=$R/$so timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/abpmc/$n/$c" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/abpmc/$n.$c.log 2>&1 || { echo "$n $c failed"; tail -5 gpurun_out/abpmc/$n.$c.log; exit 1; }
  done
done
echo ALLDONE
