#!/bin/bash
# Every BASELINE config on the final round-5 tree (one box), TF/s beside img/s.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash scripts/gpu_r5_configs.sh "16 32 64 128" "8 12 16" || exit 1
