#!/bin/bash
# Per-launch A/B of two executor option sets (tools/layer_times.py, one stream, batch 1024,
# twice each, min over runs): bash scripts/gpu_r4_lt.sh "<UNET_ENGINE base>" "<UNET_ENGINE new>" [bench args]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/lt4; mkdir -p $o
A=${1:-}; B=${2:-}; shift 2 || shift $#
for r in 1 2; do
  for tag in base new; do
    v=$A; [ $tag = new ] && v=$B
    UNET_ENGINE="fwd_streams=1${v:+,$v}" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 "$@" \
      --out $o/${tag}_$r.md > $o/${tag}_$r.log 2>&1 || { echo "layer_times $v rc=$?"; tail -20 $o/${tag}_$r.log; exit 1; }
    head -3 $o/${tag}_$r.md | tail -1
  done
done
python tools/ab_compare.py $o/base_1.md $o/base_2.md -- $o/new_1.md $o/new_2.md > $o/compare.md
head -100 $o/compare.md
