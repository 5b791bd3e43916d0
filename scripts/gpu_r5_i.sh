#!/bin/bash
# Round 5 check I: kernel profile of the native fp32 step (which f32 kernels bound it).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5i; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/f32prof -o run -- \
  python bench.py --dtype fp32 --per_gpu_batch 128 --steps 3 --warmup 1 > $o/f32prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -20 $o/f32prof.log; exit 1; }
f=$(find $o/f32prof -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
tot = collections.Counter(); cnt = collections.Counter()
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k = r["Kernel_Name"][:70]
    tot[k] += d; cnt[k] += 1
T = sum(tot.values())
print("total kernel ms (4 steps): %.1f" % (T / 1e6))
for k, v in tot.most_common(12):
    print("%8.2f ms %5d  %s" % (v / 1e6, cnt[k], k))
PY
python - "$f" > $o/f32_launches.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = len(rows) // 4
for r in rows[-n:]:
    print("%9.1f us  grid %s  %s" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
          r.get("Grid_Size", r.get("Grid_Size_X", "")), r["Kernel_Name"][:60]))
PY
sort -rn $o/f32_launches.txt | head -30
