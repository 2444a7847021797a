#!/bin/bash
# GPU-box script: tests, smoke, kernel sweep, bench, rocprofv3 profile.
# Run from the repo root. Each GPU step bounded; stop at the first failure.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail gpurun_out/smoke.log; exit 1; }
if [ "${KBENCH:-1}" = "1" ]; then
  timeout -k 10 600 python tools/kbench.py > gpurun_out/kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/kbench.log; exit 1; }
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench.err | tail -30; exit 1; }
head -c 700 gpurun_out/bench.json; echo
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  # roctx-renamed kernels: one stats row per hot-path call site (USF_ROCTX=1)
  export USF_ROCTX=1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --kernel-rename --marker-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu-baseline --no-replay > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/bench_prof.err; exit 1; }
  unset USF_ROCTX
  python tools/roofline_check.py gpurun_out/bench_prof.json gpurun_out/prof/run_kernel_stats.csv gpurun_out/bench.json > gpurun_out/roofline_check.json || exit 1
fi
echo ALLDONE
