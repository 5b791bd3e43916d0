#!/bin/bash
# Same-box A/B of the working tree against ab_base/ (scripts/ab_base.sh): per-launch
# layer times, interleaved new / base / new / base, plus one bench each.
#   bash scripts/gpu_ab.sh [layer_times args...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
out=$(pwd)/gpurun_out
for k in 1 2; do
  timeout -k 10 180 python tools/layer_times.py "$@" --out $out/ab_new_$k.md > /dev/null 2>&1 || exit $?
  (cd ab_base && timeout -k 10 180 python tools/layer_times.py "$@" --out $out/ab_base_$k.md > /dev/null 2>&1) || exit $?
done
timeout -k 10 180 python bench.py > $out/ab_bench_new.log 2>&1 || exit $?
(cd ab_base && timeout -k 10 180 python bench.py > $out/ab_bench_base.log 2>&1) || exit $?
python tools/ab_compare.py $out/ab_base_1.md $out/ab_base_2.md -- $out/ab_new_1.md $out/ab_new_2.md > $out/ab_summary.md
grep -h metric $out/ab_bench_base.log $out/ab_bench_new.log | cut -c1-160
head -5 $out/ab_summary.md
