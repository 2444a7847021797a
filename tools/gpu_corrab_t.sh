#!/bin/bash
# Correlation backward A/B timings (leaky sites + SURVEY configs) over the lib/ab builds.
set -o pipefail
CORRAB_OPS=leaky,bwd bash tools/gpu_corrab.sh > gpurun_out/ab_t.log 2>&1 || { tail -20 gpurun_out/ab_t.log; exit 1; }
grep -h "corr_bwd" gpurun_out/ab/lib_*.log
