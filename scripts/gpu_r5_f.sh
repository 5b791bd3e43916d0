#!/bin/bash
# Round 5 check F: GPU suite + headline bench + profile after the generic-wgrad store,
# wgrad reduction, tconv_fwd staging and first-layer wgrad reduction conflict fixes; and a
# kernel profile of the ATen fp32 upsampling-decoder step (70 img/s in run E).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5f; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|worst|vs float64" $o/tests.log | tail -8
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
[ $rc -eq 1 ] && grep -E "^FAILED|Error" $o/tests.log | head -20
timeout -k 10 240 python bench.py > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
grep '^{' $o/bench.log | cut -c1-200
bash scripts/gpu_profile.sh r5f > $o/profile.log 2>&1 || { echo "profile rc=$?"; tail -20 $o/profile.log; exit 1; }
head -3 gpurun_out/prof_r5f/layer_times.md | tail -1
awk -F'|' 'NR<=2 || $7+0 > 5 {print}' gpurun_out/prof_r5f/pmc_table.md
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/aten_ups -o run -- \
  python train.py --synthetic --use_upsampling --in_channels 1 --img_size 128 --batch_size 256 \
  --synthetic_train 512 --synthetic_test 256 --steps 3 --log_every 1 --no_checkpoint --noexport --noprogress \
  --backend torch --dtype fp32 > $o/aten_ups.log 2>&1 || { echo "aten prof rc=$?"; tail -20 $o/aten_ups.log; exit 1; }
f=$(find $o/aten_ups -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("ATen ups fp32: total kernel ms %.1f" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%8.1f ms %5s  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], r["Name"][:110]))
PY
