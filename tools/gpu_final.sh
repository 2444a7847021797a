#!/bin/bash
# Round evidence on the GPU box: -m gpu tests, smoke, PMC traffic passes (FETCH/WRITE) -> profiles/<TAG>_pmc_traffic.json
# (read by bench.py's roofline.traffic), the bench line, and the rocprofv3 per-site stats + roofline check.
# Usage: TAG=r04_v3 bash tools/gpu_final.sh   (run from the repo root; outputs under gpurun_out/;
# afterwards copy gpurun_out/<TAG>_pmc_traffic.json, bench.json, prof/run_kernel_stats.csv and
# roofline_check.json into profiles/ -- only gpurun_out/ comes back from the box)
set -o pipefail
R=$(pwd); TAG=${TAG:-rNN}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
PASSES="3 4" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc > gpurun_out/${TAG}_pmc_traffic.json || exit 1
cp gpurun_out/${TAG}_pmc_traffic.json profiles/ || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; grep -v "MIOpen(HIP): Warning" gpurun_out/bench.err | tail -30; exit 1; }
head -c 600 gpurun_out/bench.json; echo
export TMPDIR=/tmp USF_ROCTX=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --kernel-rename --marker-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu-baseline --no-replay > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof.err; exit 1; }
unset USF_ROCTX
python tools/roofline_check.py gpurun_out/bench_prof.json gpurun_out/prof/run_kernel_stats.csv gpurun_out/bench.json > gpurun_out/roofline_check.json || exit 1
echo ALLDONE
