#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -k "variant or golden" > gpurun_out/pytest_variants.log 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/pytest_variants.log; exit 1; }
tail -2 gpurun_out/pytest_variants.log
timeout -k 10 600 python tools/kbench.py > gpurun_out/kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/kbench.log; exit 1; }
echo done
