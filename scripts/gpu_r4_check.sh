#!/bin/bash
# Round-4 check of the current tree: full GPU suite (logs gradient-parity numbers to
# gpurun_out/parity.jsonl), smoke(), the headline + normalised-config benches, and the
# upsampling-decoder Dice parity pair (3 seeds).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
# heartbeat for the runner's silence watchdog while a single long test runs (every GPU
# step below has its own time limit); stopped on exit
( while sleep 60; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r4_suite.log 2>&1 || { echo "suite rc=$?"; tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -3 gpurun_out/r4_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
for args in "" "--norm batch --steps 10 --warmup 3" "--norm group --dtype fp16 --steps 10 --warmup 3" "--use_upsampling --in_channels 1 --steps 10 --warmup 3"; do
  timeout -k 10 240 python bench.py $args > gpurun_out/r4_b.log 2>&1 || { echo "bench $args rc=$?"; tail -20 gpurun_out/r4_b.log; exit 1; }
  grep metric gpurun_out/r4_b.log >> gpurun_out/r4_benches.jsonl
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r4_b.log') if l.startswith('{')][0]); print(d['config']['model'], d['value'], d['ms_per_step'], d.get('train_dice_last_batch'))"
done
[ "${SKIP_DICE:-0}" = 1 ] && exit 0
PAIRS=ups timeout -k 10 1200 bash scripts/gpu_dice_parity.sh 300 1 2 3 > gpurun_out/r4_dice.log 2>&1 || { echo "dice rc=$?"; tail -20 gpurun_out/r4_dice.log; exit 1; }
tail -8 gpurun_out/dice_parity.md
