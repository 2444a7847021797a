#!/bin/bash
# correlation backward: ring loop check -- parity, sweep of the default and the 4-image ring
# at all seven sites, and the bench line (in-step per-site times)
set -o pipefail
mkdir -p gpurun_out/br
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_corr_cat.py > gpurun_out/br/tests.log 2>&1 || { tail -30 gpurun_out/br/tests.log; exit 1; }
tail -2 gpurun_out/br/tests.log
timeout -k 10 400 python -u tools/corrsweep.py --op bwd --variants=-1,4 --out gpurun_out/br/bwd4.json > gpurun_out/br/bwd4.log 2>&1 || { tail -20 gpurun_out/br/bwd4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/br/bwd4.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/br/bench2.json 2> gpurun_out/br/bench.err || { grep -v "MIOpen(HIP): Warning" gpurun_out/br/bench.err | tail -30; exit 1; }
echo BRDONE
