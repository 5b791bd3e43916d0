#!/bin/bash
# Round 5 check AA: halo row carry in the persistent window -- equality tests, the GPU suite,
# same-box A/B against ab_base/ (HEAD without the carry): headline, 512^2 b32, BN.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5aa; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
for args in "--steps 20 --warmup 5" "--img_size 512 --in_channels 1 --per_gpu_batch 32 --steps 8 --warmup 3" "--norm batch --steps 10 --warmup 3"; do
  for rep in 1 2; do
    for t in base new; do
      d=.; [ $t = base ] && d=ab_base
      (cd $d && timeout -k 10 240 python bench.py $args) > $o/b.log 2>&1 || { echo "bench [$t $args] rc=$?"; tail -5 $o/b.log; exit 1; }
      echo "[$args] $t $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
