#!/bin/bash
# Forward tile-variant sweep (usf_set_variant(0, v)) at the decoder sites and SURVEY configs.
set -o pipefail
mkdir -p gpurun_out/fwdsweep
for v in -1 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python tools/corrab.py --ops fwd --fwd-variant $v --out gpurun_out/fwdsweep/v$v.json > gpurun_out/fwdsweep/v$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/fwdsweep/v$v.log; exit 1; }
done
python - <<'PY'
import json
rows={}
for v in range(-1,8):
    for r in json.load(open(f"gpurun_out/fwdsweep/v{v}.json")):
        rows.setdefault(tuple(r["shape"]),{})[v]=(r["us"], r.get("maxerr"))
for k,d in rows.items(): print(k, {v:d[v][0] for v in d}, "maxerr", max((e or 0) for _,e in d.values()))
PY
echo ALLDONE
