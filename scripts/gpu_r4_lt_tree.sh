#!/bin/bash
# Per-launch A/B of the working tree against ab_base/ (scripts/ab_base.sh <rev>): tools/layer_times.py
# on one stream at batch 1024, twice each, min over runs -> gpurun_out/lt4t/compare.md
set -o pipefail
export TMPDIR=/tmp
o=$PWD/gpurun_out/lt4t; mkdir -p $o
for r in 1 2; do
  for tag in base new; do
    d=.; [ $tag = base ] && d=ab_base
    (cd $d && UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 "$@" \
      --out $o/${tag}_$r.md) > $o/${tag}_$r.log 2>&1 || { echo "layer_times $tag rc=$?"; tail -20 $o/${tag}_$r.log; exit 1; }
    head -3 $o/${tag}_$r.md | tail -1
  done
done
python tools/ab_compare.py $o/base_1.md $o/base_2.md -- $o/new_1.md $o/new_2.md > $o/compare.md
head -100 $o/compare.md
