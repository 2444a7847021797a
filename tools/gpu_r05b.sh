#!/bin/bash
# Round-5 second box pass (outputs under gpurun_out/r05b/): persistent vs per-call
# warp/occ timing, the photometric step-counter handshake A/B (USF_PHOTO_FLAGS=1,
# lib_photoflags) with parity of both, and the Sintel mask-feature bench.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u tools/persist_ab.py --out $O/persist_ab.json > $O/persist_ab.log 2>&1 || { tail -20 $O/persist_ab.log; exit 1; }
timeout -k 10 600 python bench.py --config sintel_mf --no-cpu-baseline > $O/sintel_mf.json 2> $O/sintel_mf.err || { grep -v MIOpen $O/sintel_mf.err | tail -20; exit 1; }
head -c 400 $O/sintel_mf.json; echo
rm -rf gpurun_out/pab
AB=unsamflow_amd/lib/ab/lib_photoflags.so timeout -k 10 900 bash tools/gpu_photo_ab.sh > $O/photo_ab.log 2>&1 || { tail -30 $O/photo_ab.log; exit 1; }
tail -1 $O/photo_ab.log; cp -r gpurun_out/pab $O/pab_flags
echo R05B_DONE
