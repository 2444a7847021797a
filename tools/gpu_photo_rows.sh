#!/bin/bash
# photometric strip kernel: GPU tests, then device times at several strip heights (USF_PHOTO_ROWS).
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 400 python -u -m pytest tests/test_gpu_photometric.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03p/pt.log 2>&1
rc=$?
tail -2 gpurun_out/r03p/pt.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
for R in ${PHOTO_ROWS:-0}; do
  if [ "$R" = 0 ]; then unset USF_PHOTO_ROWS; else export USF_PHOTO_ROWS=$R; fi
  timeout -k 10 240 python tools/photoab.py --variant 0 --out gpurun_out/r03p/rows_$R.json > gpurun_out/r03p/rows_$R.log 2>&1 || { echo "rows $R failed"; tail gpurun_out/r03p/rows_$R.log; exit 1; }
  echo "== rows $R"; grep -v amdgpu.ids gpurun_out/r03p/rows_$R.log
done
