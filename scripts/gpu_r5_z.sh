#!/bin/bash
# Round 5 check Z: end-of-round evidence on the current tree -- every BASELINE config (+ 512^2 /
# 3D batch sweeps, fp32 native vs ATen), headline kernel stats / per-launch times / PMC passes,
# per-launch times of 512^2 b32, 3D b8 and the BN step.
set -o pipefail
export TMPDIR=/tmp
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash scripts/gpu_r5_configs.sh "16 32 64 128" "8 12 16" || exit 1
bash scripts/gpu_profile.sh r5z > gpurun_out/prof_r5z.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/prof_r5z.log; exit 1; }
head -3 gpurun_out/prof_r5z/layer_times.md | tail -1
o=gpurun_out/prof_r5z
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 --reps 5 \
  --out $o/layer_times_s512_b32.md > $o/lt512.log 2>&1 || { echo "lt512 rc=$?"; tail -20 $o/lt512.log; exit 1; }
head -3 $o/layer_times_s512_b32.md | tail -1
timeout -k 10 300 python tools/layer_times.py --dims 3 --batch 8 --img 128 --reps 3 \
  --out $o/layer_times_3d_b8.md > $o/lt3d.log 2>&1 || { echo "lt3d rc=$?"; tail -20 $o/lt3d.log; exit 1; }
head -3 $o/layer_times_3d_b8.md | tail -1
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out $o/layer_times_bn.md > $o/ltbn.log 2>&1 || { echo "ltbn rc=$?"; tail -20 $o/ltbn.log; exit 1; }
head -3 $o/layer_times_bn.md | tail -1
