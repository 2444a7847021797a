#!/bin/bash
# Round evidence on the GPU box (repo root), everything for one TAG:
#  1. -m gpu tests and smoke();
#  2. PMC FETCH/WRITE passes over tools/kprof.py -> gpurun_out/<TAG>_pmc_traffic.json (per launch and per
#     kernel, stamped with the library's build id), copied into profiles/ on the box so the bench below
#     reports roofline.traffic from THIS build (bench.py refuses a summary of another build);
#  3. the bench line -> gpurun_out/<TAG>_bench.json;
#  4. rocprofv3 --kernel-trace --stats of the bench step, per call site (roctx ranges, --kernel-rename)
#     -> gpurun_out/<TAG>_prof/, and per kernel (no rename) -> gpurun_out/<TAG>_prof_raw/;
#  5. tools/roofline_check.py: the roofline site's rocprof mean next to the bench's in-step mean.
# Usage: TAG=r06_final bash tools/gpu_final.sh ; afterwards copy the gpurun_out/<TAG>_* summaries into profiles/
set -o pipefail
R=$(pwd); TAG=${TAG:-rNN}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest_gpu.log; tail -3 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
PASSES="3 4" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc > gpurun_out/${TAG}_pmc_traffic.json || exit 1
cp gpurun_out/${TAG}_pmc_traffic.json profiles/ || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; grep -v "MIOpen(HIP): Warning" gpurun_out/${TAG}_bench.err | tail -30; exit 1; }
head -c 600 gpurun_out/${TAG}_bench.json; echo
export TMPDIR=/tmp USF_ROCTX=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --kernel-rename --marker-trace --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu-baseline --no-replay > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_bench_prof.err || { echo "rocprof failed"; tail -20 gpurun_out/${TAG}_bench_prof.err; exit 1; }
unset USF_ROCTX
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_raw" -o run -- python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu-baseline --no-replay > gpurun_out/${TAG}_bench_prof_raw.json 2> gpurun_out/${TAG}_bench_prof_raw.err || { echo "rocprof raw failed"; tail -20 gpurun_out/${TAG}_bench_prof_raw.err; exit 1; }
python tools/roofline_check.py gpurun_out/${TAG}_bench_prof.json gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_roofline_check.json || exit 1
echo ALLDONE
