#!/bin/bash
# Round 5 check R: same-box interleaved A/B of executor options on the headline step.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5r; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
for rep in 1 2; do
  for opt in "" "dw_fuse=0" "wg_target=384" "wg_target=768" "fwd_offset=4" "fwd_offset=9" "tconv_onload=0" "dw_wgs=1024"; do
    UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 \
      || { echo "bench [$opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "rep $rep [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
