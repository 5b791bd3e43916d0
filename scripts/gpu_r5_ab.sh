#!/bin/bash
# Round 5 check AB: persistent tconv-on-load window (conv9a forward) -- equality tests, the GPU
# suite, same-box A/B against ab_base/ (HEAD without it), per-launch times.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ab; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tconv_fused.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
for rep in 1 2 3; do
  for t in base new; do
    d=.; [ $t = base ] && d=ab_base
    (cd $d && timeout -k 10 240 python bench.py --steps 20 --warmup 5) > $o/b.log 2>&1 || { echo "bench [$t] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "$t $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --reps 5 \
  --out $o/layer_times.md > $o/lt.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt.log; exit 1; }
head -3 $o/layer_times.md | tail -1
grep -E "fwd:conv9a|fwd:conv1b|fwd:conv9b" $o/layer_times.md
