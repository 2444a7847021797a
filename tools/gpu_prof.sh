#!/bin/bash
# Per-kernel evidence for a subset of sites on the GPU box (repo root):
# FETCH/WRITE PMC passes over tools/kprof.py -> gpurun_out/<TAG>_pmc_traffic.json
# (per launch and per kernel, stamped with the build id), and a rocprofv3
# --kernel-trace --stats run of the same launches (KPROF_N=20 each) ->
# gpurun_out/<TAG>_kstats/run_kernel_stats.csv (per kernel, not per site).
# Usage: TAG=r06_x KPROF_OPS=warp_bwd,occ_bwd bash tools/gpu_prof.sh
set -o pipefail
R=$(pwd); TAG=${TAG:-rNN}; export TMPDIR=/tmp
mkdir -p gpurun_out
PASSES="3 4" timeout -k 10 600 bash tools/gpu_pmc.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc > gpurun_out/${TAG}_pmc_traffic.json || exit 1
KPROF_N=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_kstats" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/${TAG}_kstats.log 2>&1 || { echo "kernel trace failed"; tail -20 gpurun_out/${TAG}_kstats.log; exit 1; }
echo ALLDONE
