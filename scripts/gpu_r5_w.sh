#!/bin/bash
# Round 5 check W: chunk-pipelined windows -- equality tests (64-wide and the 128-wide 2D / 3D
# variant), same-box A/B on the headline, 3D and 512^2 steps, 3D kernel stats.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5w; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win_cp.py tests/test_gpu_win_pf.py \
  > $o/t.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|assert" $o/t.log | head -20; exit 1; }
tail -1 $o/t.log
ab() {   # ab <label> <bench args> -- <opts...>
  local lab=$1 args=$2; shift 2
  for opt in "$@"; do
    UNET_ENGINE="$opt" timeout -k 10 240 python bench.py $args > $o/b.log 2>&1 \
      || { echo "bench [$lab $opt] rc=$?"; tail -5 $o/b.log; exit 1; }
    echo "[$lab] [$opt] $(grep '^{' $o/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
}
for rep in 1 2; do
  ab head "--steps 20 --warmup 5" "win_cp=0" "win_cp=1" "win_cp=2"
  ab 3d "--dims 3 --per_gpu_batch 8 --steps 5 --warmup 2" "win_cp=1" "win_cp=2"
done
ab s512 "--img_size 512 --in_channels 1 --per_gpu_batch 32 --steps 5 --warmup 2" "win_cp=1" "win_cp=2"
cd /tmp
UNET_ENGINE=win_cp=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof3d -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --dims 3 --per_gpu_batch 8 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$o/prof3d.log 2>&1 \
  || { echo "prof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$o/prof3d.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$o/prof3d -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print("%-110s %6s %10.1f %6s" % (r["Name"][:110], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"][:5]))
PY
