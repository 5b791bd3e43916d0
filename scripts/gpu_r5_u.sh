#!/bin/bash
# Round 5 check U: same-box A/B of options around win_pf (dw_fuse off -> conv1b's data gradient
# on the persistent window; windows per workgroup; forward stream offset).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5u; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
for rep in 1 2; do
  for opt in "" "dw_fuse=0" "win_pf=4" "win_pf=12" "fwd_offset=4" "fwd_offset=8"; do
    UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 \
      || { echo "bench [$opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "rep $rep [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
