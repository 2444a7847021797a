#!/bin/bash
# Time A/B builds of the library (tools/ab_build.py) with the kernel sweep, one process each.
set -o pipefail
mkdir -p gpurun_out/ab
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  USF_LIB=$R$(pwd)/$so timeout -k 10 300 python tools/kbench.py --ops "${AB_OPS:-corr_fwd,corr_bwd}" --out gpurun_out/ab/$n.json > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail gpurun_out/ab/$n.log; exit 1; }
done
echo ALLDONE
