#!/bin/bash
# Round 5 check A: the new direct statistics-kernel tests, then every config.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm_fused.py -x -q --timeout 120 --timeout-method thread \
  -k "bn_stats or gn_stats" > gpurun_out/r5_stats_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r5_stats_tests.log; exit 1; }
tail -2 gpurun_out/r5_stats_tests.log
bash scripts/gpu_r5_configs.sh
