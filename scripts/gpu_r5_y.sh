#!/bin/bash
# Round 5 check Y: normalise-on-load in the persistent window (norm configs' level-1 convs) --
# equality tests, the GPU suite, same-box A/B on the BN / GN steps.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5y; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
ab() {
  local lab=$1 args=$2; shift 2
  for opt in "$@"; do
    UNET_ENGINE="$opt" timeout -k 10 240 python bench.py $args > $o/b.log 2>&1 \
      || { echo "bench [$lab $opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "[$lab] [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
}
for rep in 1 2; do
  ab bn "--norm batch --steps 10 --warmup 3" "win_pf=0" "win_pf=8"
  ab gn16 "--norm group --dtype fp16 --steps 10 --warmup 3" "win_pf=0" "win_pf=8"
done
