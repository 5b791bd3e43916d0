#!/bin/bash
# Fused Conv+BN/GN check on one GPU box: fused-epilogue kernel tests, kernel + model
# tests, then the BN / GN-fp16 side-config benches and the headline (sanity).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
val() { python -c "import json,sys; [print(sys.argv[1], json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open(sys.argv[2]) if l.startswith('{')]" "$1" "$2"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_norm_fused.py tests/test_gpu_kernels.py tests/test_gpu_model.py \
  -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_norm.log 2>&1 || { tail -60 gpurun_out/pytest_norm.log; exit 1; }
tail -3 gpurun_out/pytest_norm.log
timeout -k 10 200 python bench.py --norm batch > gpurun_out/bench_bn.log 2>&1 || exit $?
val bn gpurun_out/bench_bn.log
timeout -k 10 200 python bench.py --norm group --dtype fp16 --per_gpu_batch 1024 --steps 10 > gpurun_out/bench_gn.log 2>&1 || exit $?
val gn_fp16_b1024 gpurun_out/bench_gn.log
timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
val headline gpurun_out/bench.log
