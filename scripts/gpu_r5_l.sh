#!/bin/bash
# Round 5 check L: the whole GPU suite (incl. the bench-shape per-layer oracle), smoke().
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5l; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|checked" $o/tests.log | tail -6
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
