#!/bin/bash
# Round 5 check J/K: fp32 path after the column-sum rewrite, the channel-sized weight-gradient
# tiles: fp32 kernel + step tests, fp32 benches (both decoders), kernel profile.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py "tests/test_gpu_cli.py" -q -s --timeout 300 \
  --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|vs float64" $o/tests.log | tail -6
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
for cfg in "" "--use_upsampling --in_channels 1"; do
  timeout -k 10 300 python bench.py --dtype fp32 --per_gpu_batch 128 --steps 5 --warmup 2 $cfg > $o/f32.log 2>&1 \
    || { echo "native fp32 rc=$?"; tail -20 $o/f32.log; exit 1; }
  echo "native fp32 [$cfg]: $(grep '^{' $o/f32.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/f32prof -o run -- \
  python bench.py --dtype fp32 --per_gpu_batch 128 --steps 3 --warmup 1 > $o/f32prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -20 $o/f32prof.log; exit 1; }
f=$(find $o/f32prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms (4 steps): %.1f" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("%8.2f ms %5s  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], r["Name"][:70]))
PY
