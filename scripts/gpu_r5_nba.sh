#!/bin/bash
# norm_bwd_apply variants (UNET_NORM_EW_VAR: unroll 4/8 x non-temporal or plain loads) x grid
# width (UNET_NORM_EW_BPS), microbenchmark at the bench's level shapes; then the norm tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/nba_micro.jsonl
for v in 0 1 2 3; do
  for b in default 16; do
    if [ "$b" = default ]; then unset UNET_NORM_EW_BPS; else export UNET_NORM_EW_BPS=$b; fi
    UNET_NORM_EW_VAR=$v timeout -k 10 120 python scripts/norm_ew_micro.py | sed "s/^{/{\"var\": $v, /" >> gpurun_out/nba_micro.jsonl || exit 1
  done
done
unset UNET_NORM_EW_BPS
for v in 1 2 3; do
  UNET_NORM_EW_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k norm_fwd_bwd -x -q --timeout 120 --timeout-method thread > gpurun_out/nba_test_$v.log 2>&1 || { tail -20 gpurun_out/nba_test_$v.log; exit 1; }
  tail -1 gpurun_out/nba_test_$v.log
done
