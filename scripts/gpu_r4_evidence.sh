#!/bin/bash
# Round-4 evidence of the current tree: one-step timelines (headline / BatchNorm / GroupNorm
# fp16), the wave-cycle stall breakdown, and the N = 1 scaling rows (plain + one-rank RCCL).
# (kernel stats + layer times + PMC table: scripts/gpu_profile.sh r4, a call of its own)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash scripts/gpu_timeline.sh r4 || exit 1
bash scripts/gpu_stall_pmc.sh r4 || exit 1
python tools/stall_table.py $(find gpurun_out/stall_r4/pmc1 -name "*.db" | head -1) > gpurun_out/stall_r4/stall_table.md || exit 1
bash scripts/gpu_scale.sh gpurun_out/scale_r4.md || exit 1
bash scripts/gpu_profile.sh r4 || exit 1
