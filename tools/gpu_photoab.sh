#!/bin/bash
# Photometric A/B: tools/photoab.py once per A/B build (tools/ab_build.py), then the
# photometric + warp GPU tests against the build named by PHOTOAB_TEST (if set).
set -o pipefail
mkdir -p gpurun_out/photoab
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  USF_LIB=$(pwd)/$so timeout -k 10 240 python tools/photoab.py --out gpurun_out/photoab/$n.json > gpurun_out/photoab/$n.log 2>&1 || { echo "$n failed"; tail gpurun_out/photoab/$n.log; exit 1; }
  echo "== $n"; cat gpurun_out/photoab/$n.log
done
if [ -n "$PHOTOAB_TEST" ]; then
  USF_LIB=$(pwd)/unsamflow_amd/lib/ab/lib_$PHOTOAB_TEST.so timeout -k 10 300 python -u -m pytest tests/test_gpu_photometric.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/photoab/pt.log 2>&1 || { tail -30 gpurun_out/photoab/pt.log; exit 1; }
  tail -1 gpurun_out/photoab/pt.log
fi
echo ALLDONE
