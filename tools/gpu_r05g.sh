#!/bin/bash
# Round-5 pass G (gpurun_out/r05g/): per-kernel durations of the persistent vs per-call warp
# backward and occlusion forms (rocprofv3 kernel trace over tools/persist_ab.py).
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof" -o run -- python3 tools/persist_ab.py --out $O/persist_ab.json > $O/persist_ab.log 2>&1 || { tail -20 $O/persist_ab.log; exit 1; }
ls -R $O/prof | head
echo R05G_DONE
