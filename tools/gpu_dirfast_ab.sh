set -o pipefail
CORRAB_OPS=leaky bash tools/gpu_corrab.sh > gpurun_out/ab_t.log 2>&1 || { tail -20 gpurun_out/ab_t.log; exit 1; }
grep -h "corr_bwd_leaky" gpurun_out/ab/lib_*.log | head -20
KPROF_OPS=corr_bwd_leaky bash tools/gpu_corrab_pmc.sh > gpurun_out/ab_p.log 2>&1 || { tail -20 gpurun_out/ab_p.log; exit 1; }
python tools/abpmc_report.py gpurun_out/abpmc corr_bwd
