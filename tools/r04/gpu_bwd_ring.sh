#!/bin/bash
# correlation backward: NB=4 ring (5) vs NB=2 at the same (512-workgroup) group count (6)
# vs the defaults, at all seven sites, two runs
set -o pipefail
mkdir -p gpurun_out/br
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "every_tile_variant or corrbig or production" > gpurun_out/br/tests.log 2>&1 || { tail -30 gpurun_out/br/tests.log; exit 1; }
tail -2 gpurun_out/br/tests.log
for i in 1 2; do
timeout -k 10 400 python -u tools/corrsweep.py --op bwd --variants=-1,0,4,5,6 --out gpurun_out/br/bwd$i.json > gpurun_out/br/bwd$i.log 2>&1 || { tail -20 gpurun_out/br/bwd$i.log; exit 1; }
done
echo BRDONE
