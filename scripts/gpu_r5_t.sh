#!/bin/bash
# Round 5 check T: win_pf (persistent prefetching level-1 windows, all epilogues + head-on-load)
# -- its tests, the whole GPU suite, smoke, a same-box A/B on the headline / BN / GN steps,
# and kernel stats of the headline step.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5t; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "pf tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|checked" $o/tests.log | tail -4
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for rep in 1 2; do
  for cfg in "" "--norm batch" "--norm group --dtype fp16"; do
    for opt in "win_pf=0" "win_pf=8"; do
      UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 $cfg > $o/b.log 2>&1 \
        || { echo "bench [$cfg $opt] rc=$?"; tail -5 $o/b.log; exit 1; }
      echo "rep $rep [$cfg] [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$o/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$o/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:40]:
    print("%-100s %6s %10.1f" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
