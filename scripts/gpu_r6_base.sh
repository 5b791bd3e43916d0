#!/bin/bash
# Round 6 start: headline / BN / GN fp16 benches + BN per-launch table on the starting tree.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6base; mkdir -p $o
for cfg in "headline:" "bn:--norm batch" "gn16:--norm group --dtype fp16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 $args > $o/$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -20 $o/$tag.log; exit 1; }
  grep '^{' $o/$tag.log
done
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch \
  --out $o/lt_bn.md > $o/lt_bn.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt_bn.log; exit 1; }
head -3 $o/lt_bn.md
