#!/bin/bash
# Photometric A/B probes (lib/ab builds), then GPU tests, smoke and the bench on the in-tree library.
set -o pipefail
bash tools/gpu_photoab.sh > gpurun_out/photoab_all.log 2>&1 || { tail -20 gpurun_out/photoab_all.log; exit 1; }
grep -h '"256, 832, "border"\|== ' gpurun_out/photoab_all.log || true
PROF=0 KBENCH=0 bash tools/gpu_round.sh || exit 1
