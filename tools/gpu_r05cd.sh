#!/bin/bash
# passes D then C in one box call
set -o pipefail
bash tools/gpu_r05d.sh && bash tools/gpu_r05c.sh
