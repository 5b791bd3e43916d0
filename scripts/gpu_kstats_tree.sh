#!/bin/bash
# rocprofv3 kernel stats of the headline bench in an exported older tree and in this one:
#   bash scripts/gpu_kstats_tree.sh <old_tree_dir> [bench args] -> gpurun_out/kst_{old,new}/prof_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
old=$1; shift
top=$(pwd)
for t in old new; do
  if [ $t = old ]; then d=$old; else d=.; fi
  o=$top/gpurun_out/kst_$t
  rm -rf $o; mkdir -p $o
  (cd $d && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o run -- \
    python bench.py --steps 5 --warmup 2 "$@") > $o/ks.log 2>&1 || exit $?
  f=$(find $o/ks -name "*kernel_stats.csv" | head -1); cp $f $o/prof_kernel_stats.csv
done
