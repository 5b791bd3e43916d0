#!/bin/bash
# Round 5 check V: chunk-pipelined 64-channel windows (win_cp) -- equality tests, the GPU
# suite, smoke, same-box A/B on the headline / BN / GN steps, per-launch times.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5v; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_win_cp.py \
  > $o/t.log 2>&1 || { echo "cp tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for rep in 1 2; do
  for cfg in "" "--norm batch" "--norm group --dtype fp16"; do
    for opt in "win_cp=0" "win_cp=1"; do
      UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 $cfg > $o/b.log 2>&1 \
        || { echo "bench [$cfg $opt] rc=$?"; tail -5 $o/b.log; exit 1; }
      echo "rep $rep [$cfg] [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --in_channels 4 --reps 5 \
  --out $o/layer_times.md > $o/lt.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt.log; exit 1; }
head -3 $o/layer_times.md | tail -1
