#!/bin/bash
# tools/gpu_photo_ab.sh: photometric pair: this tree's library vs an A/B build (AB=path), parity of both, then
# tools/photoab.py alternating, two runs each
set -o pipefail
mkdir -p gpurun_out/pab
AB=${AB:-unsamflow_amd/lib/ab/lib_pairs1.so}
for L in main ab; do
  if [ $L = main ]; then unset USF_LIB; else export USF_LIB=$AB; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_photometric.py > gpurun_out/pab/tests_$L.log 2>&1 || { tail -30 gpurun_out/pab/tests_$L.log; exit 1; }
  tail -1 gpurun_out/pab/tests_$L.log
done
for i in 1 2; do
  for L in main ab; do
    if [ $L = main ]; then unset USF_LIB; else export USF_LIB=$AB; fi
    timeout -k 10 200 python -u tools/photoab.py --out gpurun_out/pab/${L}$i.json > gpurun_out/pab/${L}$i.log 2>&1 || { tail -20 gpurun_out/pab/${L}$i.log; exit 1; }
  done
done
unset USF_LIB
echo PABDONE
