#!/bin/bash
# Forward: all-rows config over channel groups (forced 10..13) vs heuristic; then
# SQ counters of the backward at the decoder sites (one rocprofv3 pass per set).
set -o pipefail
mkdir -p gpurun_out/fg gpurun_out/sqpmc
for v in -1 10 11 12 13; do
timeout -k 10 200 python tools/corrab.py --ops fwd --fwd-variant $v --out gpurun_out/fg/fwd$v.json > gpurun_out/fg/fwd$v.log 2>&1 || { tail gpurun_out/fg/fwd$v.log; exit 1; }
done
python - <<'PY'
import json
rows={}
for v in (-1,10,11,12,13):
    for r in json.load(open(f"gpurun_out/fg/fwd{v}.json")): rows.setdefault(tuple(r["shape"]),{})[v]=(r["us"], r.get("maxerr"))
for k,d in rows.items(): print(k, {n:v[0] for n,v in d.items()}, "maxerr", max((v[1] or 0) for v in d.values()))
PY
export TMPDIR=/tmp KPROF_OPS=corr_bwd_leaky,corr_fwd KPROF_N=3
R=$(pwd)
i=0
for set in "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,SQ_INSTS_LDS,SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VMEM,SQ_INSTS_VMEM,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_INSTS_SALU,SQ_ACTIVE_INST_SCA" \
           "TA_BUSY_avr,TA_FLAT_READ_WAVEFRONTS_sum,GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --kernel-trace --output-format csv -d "$R/gpurun_out/sqpmc/p$i" -o run -- python3 "$R/tools/kprof.py" > gpurun_out/sqpmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/sqpmc/p$i.log; }
done
echo ALLDONE
