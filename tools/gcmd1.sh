set -o pipefail
mkdir -p gpurun_out
for args in "bwd 16 32 64 208" "bwd 8 32 64 208" "bwd 8 128 32 104" "fwd 8 128 32 104" "fwd 16 32 64 208"; do
  timeout -k 5 60 ./tools/probes/corr_trace $args >> gpurun_out/corr_trace.txt 2>&1 || { echo "trace failed: $args"; exit 1; }
done
PASSES="1 2" bash tools/gpu_pmc_corr.sh > gpurun_out/pmc_corr.log 2>&1 || { tail -30 gpurun_out/pmc_corr.log; exit 1; }
tail -40 gpurun_out/pmc_corr.log
