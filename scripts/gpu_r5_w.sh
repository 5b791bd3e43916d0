#!/bin/bash
# Round 5 check W: win_cp restricted to 64-wide rows (tests + same-box A/B), and kernel
# stats of the 3D step (which kernels the 3D level-1 data gradients run).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5w; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win_cp.py tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
for rep in 1 2 3; do
  for opt in "win_cp=0" "win_cp=1"; do
    UNET_ENGINE="$opt" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 \
      || { echo "bench [$opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "rep $rep [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof3d -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --dims 3 --per_gpu_batch 8 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$o/prof3d.log 2>&1 \
  || { echo "prof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$o/prof3d.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$o/prof3d -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print("%-110s %6s %10.1f %6s" % (r["Name"][:110], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"][:5]))
PY
