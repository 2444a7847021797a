#!/bin/bash
# Warp backward check: its GPU tests, the A/B timing of the default path at the
# decoder sites (tools/warpab.py) with the persistent workspace and with
# per-call filled ones, and rocprofv3 kernel traces at L4.
set -o pipefail
mkdir -p gpurun_out/wchk
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "warp" tests/test_gpu_graph_replay.py > gpurun_out/wchk/tests.log 2>&1 \
  || { tail -40 gpurun_out/wchk/tests.log; exit 1; }
tail -3 gpurun_out/wchk/tests.log
for p in 1 0; do
  USF_WARP_PERSIST=$p timeout -k 10 300 python tools/warpab.py --variants=-1 --out gpurun_out/wchk/warpab_p$p.json > gpurun_out/wchk/warpab_p$p.log 2>&1 \
    || { tail -20 gpurun_out/wchk/warpab_p$p.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
for f in pm2 shift; do
  KPROF_N=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wchk/prof_$f -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/warp_kprof2.py $f > $GRAFT_REPO_ROOT/gpurun_out/wchk/prof_$f.log 2>&1 || exit 1
done
echo WCHKDONE
