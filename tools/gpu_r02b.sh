#!/bin/bash
# A/B: early stage-0 DMA (lib/ab builds), then 16x16-tile candidates with the main library.
set -o pipefail
mkdir -p gpurun_out/ab; bash tools/gpu_corrab.sh > gpurun_out/ab/corrab.log 2>&1 || { tail -20 gpurun_out/ab/corrab.log; exit 1; }
mkdir -p gpurun_out/t16
timeout -k 10 200 python tools/corrab.py --ops bwd,leaky --bwd-variant 4 --out gpurun_out/t16/bwd4.json > gpurun_out/t16/bwd4.log 2>&1 || { tail gpurun_out/t16/bwd4.log; exit 1; }
timeout -k 10 200 python tools/corrab.py --ops bwd,leaky --bwd-variant 0 --out gpurun_out/t16/bwd0.json > gpurun_out/t16/bwd0.log 2>&1 || { tail gpurun_out/t16/bwd0.log; exit 1; }
for v in 2 4 8 9; do
timeout -k 10 200 python tools/corrab.py --ops fwd --fwd-variant $v --out gpurun_out/t16/fwd$v.json > gpurun_out/t16/fwd$v.log 2>&1 || { tail gpurun_out/t16/fwd$v.log; exit 1; }
done
python - <<'PY'
import json
def show(tag, files):
    rows={}
    for n,f in files:
        for r in json.load(open(f)): rows.setdefault((r["op"],tuple(r["shape"])),{})[n]=(r["us"], r.get("maxerr"))
    print("==", tag)
    for k,d in rows.items(): print(k, {n:v[0] for n,v in d.items()}, "maxerr", max((v[1] or 0) for v in d.values()))
show("early", [("early0","gpurun_out/ab/lib_early0.json"),("early1","gpurun_out/ab/lib_early1.json")])
show("bwd tiles", [("v0","gpurun_out/t16/bwd0.json"),("v4_16x16","gpurun_out/t16/bwd4.json")])
show("fwd tiles", [(f"v{v}",f"gpurun_out/t16/fwd{v}.json") for v in (2,4,8,9)])
PY
echo ALLDONE
