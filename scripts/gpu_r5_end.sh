#!/bin/bash
# End of the round-5 re-entry session: the round-end commands on the final tree (every GPU
# test, smoke(), the 1-GPU headline bench) and rocprofv3 kernel statistics of the BatchNorm
# and GroupNorm fp16 steps.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 180 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep metric gpurun_out/bench.log
for cfg in bn gn16; do
  if [ $cfg = bn ]; then args="--norm batch"; else args="--norm group --dtype fp16"; fi
  o=gpurun_out/prof_end_$cfg; rm -rf $o; mkdir -p $o
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o run -- \
    python bench.py $args --steps 5 --warmup 2 > $o/ks.log 2>&1 || { echo "prof $cfg rc=$?"; tail -20 $o/ks.log; exit 1; }
  f=$(find $o/ks -name "*kernel_stats.csv" | head -1); cp $f $o/prof_kernel_stats.csv
  python tools/prof_summary.py $o 7 "bench.py 2D 128x128x4 b1024 $args (round 5 final tree)" > $o/kernel_stats.md || exit 1
  head -8 $o/kernel_stats.md
done
