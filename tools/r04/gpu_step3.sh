#!/bin/bash
# correlation backward: DPP-window variants (usf_set_variant(1, 4 / 5)) parity, then A/B timing vs the default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_corr_cat.py -k "every_tile_variant or dpp_window or production_backward" > gpurun_out/s3_tests.log 2>&1 || { tail -40 gpurun_out/s3_tests.log; exit 1; }
tail -3 gpurun_out/s3_tests.log
for v in -1 4 5; do
  timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --bwd-variant $v --out gpurun_out/s3_corrab_v$v.json > gpurun_out/s3_corrab_v$v.log 2>&1 || { tail -20 gpurun_out/s3_corrab_v$v.log; exit 1; }
done
grep -h '"op"' gpurun_out/s3_corrab_v*.log | head -60
USF_LIB=unsamflow_amd/lib/ab/lib_dirfast.so timeout -k 10 300 python -u tools/corrab.py --ops leaky,bwd --out gpurun_out/s3_corrab_dirfast.json > gpurun_out/s3_corrab_dirfast.log 2>&1 || { tail -20 gpurun_out/s3_corrab_dirfast.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_wprof -o run -- python3 tools/warpab.py --variants 8,6 --out gpurun_out/s3_warpab_prof.json > gpurun_out/s3_wprof.log 2>&1 || { tail -20 gpurun_out/s3_wprof.log; exit 1; }
echo S3DONE
