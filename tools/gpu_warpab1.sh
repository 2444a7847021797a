#!/bin/bash
# tools/warpab.py with the main library: default path vs the atomic scatter (variant 0... per --variants)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/warpab.py --variants=${WARPAB_VARIANTS:--1} --out gpurun_out/warpab1.json > gpurun_out/warpab1.log 2>&1 || { tail gpurun_out/warpab1.log; exit 1; }
python - <<'PY'
import json
d = {}
for r in json.load(open("gpurun_out/warpab1.json")):
    d.setdefault((tuple(r["shape"]), r["flow"]), {})[r["variant"]] = r["us"]
for k, v in d.items(): print(k, v)
PY
echo ALLDONE
