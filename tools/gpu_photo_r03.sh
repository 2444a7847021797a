#!/bin/bash
# Round 3: photometric strip kernel -- GPU tests, A/B timing strip vs tile, PMC of the strip kernel.
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 400 python -u -m pytest tests/test_gpu_photometric.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03p/pt.log 2>&1
rc=$?
tail -4 gpurun_out/r03p/pt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
for v in ${PHOTO_VARIANTS:-0 1}; do
  timeout -k 10 240 python tools/photoab.py --variant $v --out gpurun_out/r03p/ab_v$v.json > gpurun_out/r03p/ab_v$v.log 2>&1 || { echo "ab $v failed"; tail gpurun_out/r03p/ab_v$v.log; exit 1; }
  echo "== variant $v"; grep -v amdgpu.ids gpurun_out/r03p/ab_v$v.log
done
if [ -n "$PHOTO_PMC" ]; then
  KPROF_OPS=photo_pair_grad bash tools/gpu_photo_prof.sh > gpurun_out/r03p/prof.log 2>&1 || { tail gpurun_out/r03p/prof.log; exit 1; }
  python tools/pmc_report.py gpurun_out/pp | grep -i photo
fi
exit $rc
