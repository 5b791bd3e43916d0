#!/bin/bash
# Round-4 start: same-box headline bench, the new CLI / multi-rank bench tests, one-step timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/r4base_bench.log 2>&1 || exit $?
grep metric gpurun_out/r4base_bench.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_cli.py \
  tests/test_gpu_dist.py -k "bench or train" > gpurun_out/r4base_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r4base_tests.log; exit 1; }
tail -5 gpurun_out/r4base_tests.log
bash scripts/gpu_timeline.sh r4base > gpurun_out/tl_r4base.log 2>&1 || { echo "timeline rc=$?"; exit 1; }
echo timeline done
