#!/bin/bash
# per-kernel split of the binned warp backward at the decoder's sites (kernel trace, no renaming)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ws
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ws/prof -o run -- python3 tools/sitebench.py --ops warp_bwd,warp_fwd,occ_bwd --out gpurun_out/ws/site.json > gpurun_out/ws/site.log 2>&1 || { tail -20 gpurun_out/ws/site.log; exit 1; }
echo WSDONE
