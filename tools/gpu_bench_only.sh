#!/bin/bash
# The driver's bench command alone (default flags), output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench.err | tail -30; exit 1; }
head -c 300 gpurun_out/bench.json; echo
echo ALLDONE
