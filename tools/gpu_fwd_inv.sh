#!/bin/bash
# Forward epilogue A/B (device times of the decoder forward + SURVEY configs), then the
# correlation GPU tests on the in-tree library.
set -o pipefail
mkdir -p gpurun_out/ab
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  USF_LIB=$(pwd)/$so timeout -k 10 300 python tools/sitebench.py --ops corr_fwd_leaky,corr_fwd --out gpurun_out/ab/$n.json > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail gpurun_out/ab/$n.log; exit 1; }
  echo "== $n"; cat gpurun_out/ab/$n.log | grep -v amdgpu.ids
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "corr or graph or harness or pwclite" --timeout 120 --timeout-method thread > gpurun_out/corr_tests.log 2>&1 || { tail -40 gpurun_out/corr_tests.log; exit 1; }
tail -2 gpurun_out/corr_tests.log
echo ALLDONE
