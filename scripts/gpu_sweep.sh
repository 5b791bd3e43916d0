#!/bin/bash
# batch-size sweep + per-launch layer times + rocprofv3 kernel stats of the headline bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 256 512 1024; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --per_gpu_batch $b > gpurun_out/bench_b$b.log 2>&1 || exit $?
done
timeout -k 10 180 python tools/layer_times.py --batch 256 --img 128 --out gpurun_out/layer_times_b256.md > /dev/null 2>&1 || exit $?
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); d=$(dirname $f); cp $f $d/prof_kernel_stats.csv
python tools/prof_summary.py $d 7 "bench.py 2D 128x128x4 b256 bf16 hip_graph" > gpurun_out/prof_summary.md
cat gpurun_out/bench_b*.log | grep metric
