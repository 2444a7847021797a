#!/bin/bash
# Forward candidates incl. the in-workgroup channel halves (CS = 2: variants 8, 9),
# then phase traces of the backward at L4 (batch 16) and SURVEY config 2.
set -o pipefail
mkdir -p gpurun_out/fwdcs
for v in -1 5 8 9; do
  timeout -k 10 200 python tools/corrab.py --ops fwd --fwd-variant $v --out gpurun_out/fwdcs/v$v.json > gpurun_out/fwdcs/v$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/fwdcs/v$v.log; exit 1; }
done
python - <<'PY'
import json
rows={}
for v in (-1,5,8,9):
    for r in json.load(open(f"gpurun_out/fwdcs/v{v}.json")):
        rows.setdefault(tuple(r["shape"]),{})[v]=(r["us"], r.get("maxerr"))
for k,d in rows.items(): print(k, {v:d[v][0] for v in d}, "maxerr", max((e or 0) for _,e in d.values()))
PY
out=gpurun_out/fwdcs/trace.txt; : > $out
for args in "bwd 16 32 64 208" "bwd 8 128 32 104" "fwd 8 128 32 104" "fwd 8 128 32 104 8"; do
  timeout -k 5 60 ./tools/probes/corr_trace $args >> $out 2>&1 || { echo "trace failed: $args"; cat $out; exit 1; }
done
cat $out
echo ALLDONE
