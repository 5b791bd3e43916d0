#!/bin/bash
# Rehearse the multi-rank bench path on a 1-GPU box: 2 ranks share the card and
# talk over gloo (RCCL refuses two ranks on one device).  Exercises rank/device
# setup, parameter broadcast, bucketed async allreduce between HIP-graph segment
# replays, the max-over-ranks timing and rank-0-only output.  Then a rocprofv3
# kernel-stats profile of the 1-GPU headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
UNET_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --per_gpu_batch 64 \
  > gpurun_out/bench_2rank_gloo.log 2>&1 || exit $?
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); d=$(dirname $f); cp $f $d/prof_kernel_stats.csv
python tools/prof_summary.py $d 7 "bench.py 2D 128x128x4 b256 bf16 hip_graph" > gpurun_out/prof_summary.md
grep metric gpurun_out/bench_2rank_gloo.log
