#!/bin/bash
# Round 5 check AC: stream options on the tree with the persistent windows (same-box A/B).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ac; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
for rep in 1 2 3; do
  for opt in ${OPTS:-"" "fwd_streams=1" "fwd_offset=3" "fwd_offset=9" "dual_stream=0"}; do
    UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 \
      || { echo "bench [$opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "rep $rep [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
