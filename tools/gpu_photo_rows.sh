#!/bin/bash
# Photometric pair at forced strip heights (USF_PHOTO_ROWS), full resolution rows of tools/photoab.py
set -o pipefail
mkdir -p gpurun_out/prow
for R in 29 22 26 32 37 29; do
  USF_PHOTO_ROWS=$R timeout -k 10 200 python -u tools/photoab.py --out gpurun_out/prow/r$R.json > gpurun_out/prow/r$R.log 2>&1 || { tail -5 gpurun_out/prow/r$R.log; exit 1; }
  echo "R=$R $(head -1 gpurun_out/prow/r$R.log | cut -c1-120)"
  grep '256, 832, "border"' gpurun_out/prow/r$R.log | head -2
done
