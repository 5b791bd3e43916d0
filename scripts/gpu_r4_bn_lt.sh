#!/bin/bash
# Per-launch times of the BatchNorm / GroupNorm steps (tools/layer_times.py, batch 1024):
# bash scripts/gpu_r4_bn_lt.sh [tag]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/bnlt${1:+_$1}; mkdir -p $o
timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out $o/bn.md > $o/bn.log 2>&1 || { echo "bn rc=$?"; tail -20 $o/bn.log; exit 1; }
head -3 $o/bn.md | tail -1
timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm group --dtype fp16 --reps 5 \
  --out $o/gn16.md > $o/gn16.log 2>&1 || { echo "gn rc=$?"; tail -20 $o/gn16.log; exit 1; }
head -3 $o/gn16.md | tail -1
