#!/bin/bash
# Correlation A/B over the lib/ab builds, compact table at the end.
set -o pipefail
mkdir -p gpurun_out/ab
bash tools/gpu_corrab.sh > gpurun_out/ab/corrab.log 2>&1 || { tail -20 gpurun_out/ab/corrab.log; exit 1; }
python - <<'PY'
import json, glob, os
libs=sorted(glob.glob("unsamflow_amd/lib/ab/lib_*.so"))
rows={}
for so in libs:
    n=os.path.basename(so)[4:-3]
    for r in json.load(open(f"gpurun_out/ab/lib_{n}.json")): rows.setdefault((r["op"],tuple(r["shape"])),{})[n]=(r["us"], r.get("maxerr"))
for k,d in rows.items(): print(k, {n:v[0] for n,v in d.items()}, "maxerr", max((v[1] or 0) for v in d.values()))
PY
echo ALLDONE
