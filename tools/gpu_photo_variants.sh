#!/bin/bash
# photometric kernels: GPU tests (default kernel), then device times per usf_set_variant(3, v).
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 400 python -u -m pytest tests/test_gpu_photometric.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03p/pt.log 2>&1
rc=$?
tail -2 gpurun_out/r03p/pt.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/r03p/pt.log | head; echo "pytest rc $rc: stop"; exit $rc; fi
for v in ${PHOTO_VARIANTS:-0 2}; do
  timeout -k 10 240 python tools/photoab.py --variant $v --out gpurun_out/r03p/var_$v.json > gpurun_out/r03p/var_$v.log 2>&1 || { echo "variant $v failed"; tail gpurun_out/r03p/var_$v.log; exit 1; }
  echo "== variant $v"; grep -v amdgpu.ids gpurun_out/r03p/var_$v.log
done
