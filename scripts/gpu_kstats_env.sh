#!/bin/bash
# rocprofv3 kernel stats of the headline bench under two settings of an env knob:
#   bash scripts/gpu_kstats_env.sh VAR A B   -> gpurun_out/kst_<VAR>_<v>/kernel_stats.md
set -o pipefail
export TMPDIR=/tmp
var=$1; shift
for v in "$@"; do
  o=gpurun_out/kst_${var}_$v
  rm -rf $o; mkdir -p $o
  env $var=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o run -- \
    python bench.py --steps 5 --warmup 2 > $o/ks.log 2>&1 || exit $?
  f=$(find $o/ks -name "*kernel_stats.csv" | head -1); cp $f $o/prof_kernel_stats.csv
  python tools/prof_summary.py $o 7 "bench.py headline, $var=$v" > $o/kernel_stats.md || exit $?
done
