#!/bin/bash
# Round evidence: GPU tests, smoke, bench, rocprofv3 per-site stats, PMC traffic passes.
set -o pipefail
R=$(pwd)
KBENCH=0 bash tools/gpu_round.sh || exit 1
PASSES="3 4" bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc > gpurun_out/pmc_traffic.json || exit 1
echo FINALDONE
