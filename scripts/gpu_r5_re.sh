#!/bin/bash
# Round 5 re-entry check: the rebuilt tree on a fresh box -- every GPU test, smoke(), the
# headline bench and the BatchNorm bench.
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
timeout -k 10 180 python bench.py --norm batch --steps 10 --warmup 3 > gpurun_out/bench_bn.log 2>&1 || exit $?
grep metric gpurun_out/bench_bn.log
for b in default 1 2 4 8 16; do
  if [ "$b" = default ]; then unset UNET_NORM_EW_BPS; else export UNET_NORM_EW_BPS=$b; fi
  timeout -k 10 120 python scripts/norm_ew_micro.py >> gpurun_out/norm_ew_micro.jsonl 2> gpurun_out/norm_ew_micro.err || { tail -5 gpurun_out/norm_ew_micro.err; exit 1; }
done
unset UNET_NORM_EW_BPS
tail -3 gpurun_out/norm_ew_micro.jsonl
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out gpurun_out/layer_times_bn.md > gpurun_out/ltbn.log 2>&1 || { echo "ltbn rc=$?"; tail -20 gpurun_out/ltbn.log; exit 1; }
head -3 gpurun_out/layer_times_bn.md | tail -1
timeout -k 10 300 python scripts/ups_parity_diag.py > gpurun_out/ups_diag.jsonl 2> gpurun_out/ups_diag.err || { tail -5 gpurun_out/ups_diag.err; exit 1; }
