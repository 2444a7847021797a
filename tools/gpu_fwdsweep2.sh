#!/bin/bash
# Forward candidates (usf_set_variant(0, v)) at the decoder sites and SURVEY configs.
set -o pipefail
mkdir -p gpurun_out/fs2
VS=${FWD_VARIANTS:--1 8 9 10 11}
for v in $VS; do
  timeout -k 10 200 python tools/corrab.py --ops fwd --fwd-variant $v --out gpurun_out/fs2/v$v.json > gpurun_out/fs2/v$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/fs2/v$v.log; exit 1; }
done
python - $VS <<'PY'
import json, sys
rows={}
for v in sys.argv[1:]:
    for r in json.load(open(f"gpurun_out/fs2/v{v}.json")):
        rows.setdefault(tuple(r["shape"]),{})[v]=(r["us"], r.get("maxerr"))
for k,d in rows.items(): print(k, {v:d[v][0] for v in d}, "maxerr", max((e or 0) for _,e in d.values()))
PY
echo ALLDONE
