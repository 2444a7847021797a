#!/bin/bash
# Correlation A/B: tools/corrab.py once per A/B build (tools/ab_build.py), one process each.
# CORRAB_ARGS passes extra arguments (e.g. --bwd-variant 1) to every run.
set -o pipefail
mkdir -p gpurun_out/ab
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  USF_LIB=$(pwd)/$so timeout -k 10 300 python tools/corrab.py --ops "${CORRAB_OPS:-fwd,bwd,leaky}" ${CORRAB_ARGS} --out gpurun_out/ab/$n.json > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail gpurun_out/ab/$n.log; exit 1; }
  echo "== $n"; cat gpurun_out/ab/$n.log
done
echo ALLDONE
