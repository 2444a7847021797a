#!/bin/bash
# Round-5 pass F (gpurun_out/r05f/): corr backward wave-priority A/Bs (lib_prio1: raised
# during the FMAs, lib_prio2: raised while issuing the next stage's DMA) and a full forward
# candidate sweep at the seven correlation sites (every usf_set_variant(0, i)).
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
for NAME in prio1 prio2; do
  rm -rf gpurun_out/bab
  OP=bwd AB=unsamflow_amd/lib/ab/lib_$NAME.so timeout -k 10 900 bash tools/gpu_corr_ab.sh > $O/ab_$NAME.log 2>&1 || { tail -30 $O/ab_$NAME.log; exit 1; }
  tail -1 $O/ab_$NAME.log; cp -r gpurun_out/bab $O/bab_$NAME
done
timeout -k 10 400 python -u tools/corrsweep.py --op fwd --out $O/fwd_all.json > $O/fwd_all.log 2>&1 || { tail -20 $O/fwd_all.log; exit 1; }
echo R05F_DONE
