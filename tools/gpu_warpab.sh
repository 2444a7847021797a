#!/bin/bash
# tools/warpab.py once per A/B build (tools/ab_build.py), one process each.
set -o pipefail
mkdir -p gpurun_out/wab
for so in unsamflow_amd/lib/ab/lib_*.so; do
  n=$(basename $so .so)
  USF_LIB=$(pwd)/$so timeout -k 10 300 python tools/warpab.py --variants=${WARPAB_VARIANTS:--1} --out gpurun_out/wab/$n.json > gpurun_out/wab/$n.log 2>&1 || { echo "$n failed"; tail gpurun_out/wab/$n.log; exit 1; }
done
python - <<'PY'
import json, glob, os
d = {}
for f in sorted(glob.glob("gpurun_out/wab/lib_*.json")):
    n = os.path.basename(f)[4:-5]
    for r in json.load(open(f)):
        d.setdefault((tuple(r["shape"]), r["flow"]), {})[f"{n}:{r['variant']}"] = r["us"]
for k, v in d.items():
    print(k, v)
PY
echo ALLDONE
