#!/bin/bash
# Round-5 third box pass (outputs under gpurun_out/r05c/): small-grid backward order
# A/B, this tree (a tile's channel groups on one XCD) vs USF_BWD_GROUP_XCD=2 (all of a
# sample-direction's tiles on one XCD, lib_sampxcd), parity of both, PMC traffic.
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
NAME=sampxcd; KOPS=corr_bwd_leaky,corr_bwd
rm -rf gpurun_out/bab
OP=bwd AB=unsamflow_amd/lib/ab/lib_$NAME.so timeout -k 10 900 bash tools/gpu_corr_ab.sh > $O/ab_$NAME.log 2>&1 || { tail -30 $O/ab_$NAME.log; exit 1; }
tail -1 $O/ab_$NAME.log; cp -r gpurun_out/bab $O/bab_$NAME
for L in main ab; do
  if [ $L = main ]; then unset USF_LIB; else export USF_LIB=unsamflow_amd/lib/ab/lib_$NAME.so; fi
  for P in FETCH_SIZE WRITE_SIZE; do
    n=3; [ $P = WRITE_SIZE ] && n=4
    KPROF_OPS=$KOPS timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$(pwd)/$O/pmc_${NAME}_$L/p$n" -o run -- python3 tools/kprof.py > $O/pmc_${NAME}_${L}_$n.log 2>&1 || { echo "pmc $L $P failed"; tail $O/pmc_${NAME}_${L}_$n.log; exit 1; }
  done
  KPROF_OPS=$KOPS python tools/pmc_traffic.py $O/pmc_${NAME}_$L > $O/traffic_${NAME}_$L.json || exit 1
done
unset USF_LIB
echo R05C_DONE
