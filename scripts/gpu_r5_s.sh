#!/bin/bash
# Round 5 check S: persistent prefetching level-1 window (win_pf) -- kernel equality tests,
# then a same-box interleaved A/B of win_pf on the headline step, then per-kernel stats.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5s; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/t.log; exit 1; }
tail -3 $o/t.log
for rep in 1 2; do
  for opt in "win_pf=0" "win_pf=16" "win_pf=8" "win_pf=32"; do
    UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 \
      || { echo "bench [$opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "rep $rep [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$o/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$o/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "conv_win" in n and ("128, 32, 512" in n or "pf" in n):
        print("%-90s %6s %10.1f" % (n[:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
