#!/bin/bash
# Round 5 check N: every BASELINE config on the current tree (scripts/gpu_r5_configs.sh).
set -o pipefail
export TMPDIR=/tmp
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash scripts/gpu_r5_configs.sh "16 32 64 128" "8 12 16"
