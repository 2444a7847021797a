#!/bin/bash
# tools/gpu_corr_ab.sh: correlation default (OP=bwd|fwd) at all seven sites: this tree's library vs an A/B build (USF_LIB),
# alternating, two runs each
set -o pipefail
mkdir -p gpurun_out/bab
AB=${AB:-unsamflow_amd/lib/ab/lib_cv2.so}
for L in main ab; do
  if [ $L = main ]; then unset USF_LIB; else export USF_LIB=$AB; fi
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_corr_cat.py > gpurun_out/bab/tests_$L.log 2>&1 || { tail -30 gpurun_out/bab/tests_$L.log; exit 1; }
  tail -1 gpurun_out/bab/tests_$L.log
done
for i in 1 2; do
  for L in main ab; do
    if [ $L = main ]; then unset USF_LIB; else export USF_LIB=$AB; fi
    timeout -k 10 300 python -u tools/corrsweep.py --op ${OP:-bwd} --variants=-1 --out gpurun_out/bab/${L}$i.json > gpurun_out/bab/${L}$i.log 2>&1 || { tail -20 gpurun_out/bab/${L}$i.log; exit 1; }
  done
done
unset USF_LIB
echo BABDONE
