#!/bin/bash
# Round 6 end: rocprofv3 kernel stats of the 3D b8 and headline steps on the final tree.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6profend; mkdir -p $o
for cfg in "d3:--dims 3 --steps 5 --warmup 2" "head:--steps 5 --warmup 2"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  rm -rf $o/$tag; mkdir -p $o/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag/ks -o run -- \
    python bench.py --hip_graph 0 $args > $o/$tag/ks.log 2>&1 || { echo "ks $tag rc=$?"; tail $o/$tag/ks.log; exit 1; }
  f=$(find $o/$tag/ks -name "*kernel_stats.csv" | head -1); cp $f $o/$tag/prof_kernel_stats.csv
  python tools/prof_summary.py $o/$tag 7 "bench.py $tag (round 6 end tree)" > $o/$tag/kernel_stats.md || exit 1
  head -4 $o/$tag/kernel_stats.md
done
