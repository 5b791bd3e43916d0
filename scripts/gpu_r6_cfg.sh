#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash scripts/gpu_r6_configs.sh "32 64 128" "8 16" || exit 1
