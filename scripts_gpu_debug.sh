#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/debug_warp.py > gpurun_out/debug_warp.log 2>&1 || { echo "debug_warp rc=$?"; cat gpurun_out/debug_warp.log | tail; exit 1; }
cat gpurun_out/debug_warp.log
USF_SYNC_CHECK=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 1 > gpurun_out/bench_sync.json 2> gpurun_out/bench_sync.err || { echo "bench_sync failed rc=$?"; grep -v "^MIOpen(HIP): Warning" gpurun_out/bench_sync.err | tail -30; exit 1; }
echo "sync bench ok"; head -c 600 gpurun_out/bench_sync.json
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; grep -v "^MIOpen(HIP): Warning" gpurun_out/bench.err | tail -30; exit 1; }
cat gpurun_out/bench.json
