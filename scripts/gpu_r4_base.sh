#!/bin/bash
# Round-4 start: same-box headline / BN / GN-fp16 benches and one-step timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/r4base_bench.log 2>&1 || exit $?
grep metric gpurun_out/r4base_bench.log
bash scripts/gpu_timeline.sh r4base > gpurun_out/tl_r4base.log 2>&1 || { echo "timeline rc=$?"; exit 1; }
echo timeline done
