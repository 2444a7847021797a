#!/bin/bash
# Round-5 first box pass (outputs under gpurun_out/r05a/): A/B of the forward edge
# order (this tree vs USF_FWD_EDGE_XCD=0, lib_fwdchunk) and of the small-grid backward
# order (vs USF_BWD_GROUP_XCD=0, lib_grpxcd0), each with parity tests and PMC traffic;
# the new persistent warp/occ tests then the whole -m gpu suite; persistent vs per-call
# timing; the Sintel mask-feature bench (SURVEY config 5 per GPU).
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
for X in fwd:fwdchunk:corr_fwd_leaky bwd:grpxcd0:corr_bwd_leaky; do
  IFS=: read OPX NAME KOPS <<< "$X"
  rm -rf gpurun_out/bab
  OP=$OPX AB=unsamflow_amd/lib/ab/lib_$NAME.so timeout -k 10 900 bash tools/gpu_corr_ab.sh > $O/ab_$NAME.log 2>&1 || { tail -30 $O/ab_$NAME.log; exit 1; }
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
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_persist.py > $O/persist_tests.log 2>&1 || { tail -40 $O/persist_tests.log; exit 1; }
tail -2 $O/persist_tests.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u tools/corrsweep.py --op bwd --variants=-1,5,6 --out $O/bwd_flags$i.json > $O/bwd_flags$i.log 2>&1 || { tail -20 $O/bwd_flags$i.log; exit 1; }
done
echo R05A_DONE
