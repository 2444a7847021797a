#!/bin/bash
# Eager PWCLite step time under MIOpen solver toggles / memory formats (each
# configuration its own process: MIOpen reads its env at init).
set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 240 python tools/graph_probe.py --eager-only --tag "$tag" $EXTRA 2>/dev/null | grep eager_ms >> gpurun_out/conv_probe.jsonl || echo "{\"tag\": \"$tag\", \"failed\": true}" >> gpurun_out/conv_probe.jsonl; }
: > gpurun_out/conv_probe.jsonl
EXTRA="" run base X=1
EXTRA="--channels-last" run nhwc X=1
EXTRA="" run no_winograd MIOPEN_DEBUG_CONV_WINOGRAD=0
EXTRA="--channels-last" run nhwc_no_winograd MIOPEN_DEBUG_CONV_WINOGRAD=0
EXTRA="" run no_direct MIOPEN_DEBUG_CONV_DIRECT=0
EXTRA="" run no_implicit_gemm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0
cat gpurun_out/conv_probe.jsonl
