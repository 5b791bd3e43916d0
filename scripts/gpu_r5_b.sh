#!/bin/bash
# Round 5 check B: 3D batch sweep, per-launch times of the 512^2 config (batch 64) and 3D.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5cfg; mkdir -p $o
SKIP_MAIN=1 bash scripts/gpu_r5_configs.sh "" "8 12 16" || { echo "configs failed"; exit 1; }
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 64 --img 512 --in_channels 1 --reps 5 \
  --out $o/lt_512_b64.md > $o/lt_512.log 2>&1 || { echo "lt512 rc=$?"; tail -20 $o/lt_512.log; exit 1; }
head -3 $o/lt_512_b64.md
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 8 --img 128 --dims 3 --reps 3 \
  --out $o/lt_3d_b8.md > $o/lt_3d.log 2>&1 || { echo "lt3d rc=$?"; tail -20 $o/lt_3d.log; exit 1; }
head -3 $o/lt_3d_b8.md
