#!/bin/bash
# Round-end style check on one GPU box: every GPU test, smoke(), the 1-GPU headline
# bench, then the 2-rank gloo rehearsal + rocprofv3 kernel stats (gpu_multirank.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 180 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep metric gpurun_out/bench.log
bash scripts/gpu_multirank.sh
