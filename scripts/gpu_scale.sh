#!/bin/bash
# Multi-GPU scaling + RCCL tuning sweep of the headline bench on ONE node, one table:
#   N = 1 / 2 / 4 / 8 ranks (torch.distributed.run, one process per GPU, RCCL over xGMI),
#   --bucket_mb 2 / 4 / 8 / 16 and NCCL_MIN_NCHANNELS unset / 16 / 32 at every N > 1,
# each line carrying the bench's comm diagnostics (per-bucket allreduce time, exposed
# communication = overlapped step - compute-only step).  N larger than the GPUs this
# box has is skipped (a 1-GPU box runs only N = 1, plus the one-rank RCCL bucket path
# via --dist_force 1).
#   bash scripts/gpu_scale.sh [out.md] [extra bench args]
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=${1:-gpurun_out/scale.md}; shift || true
mkdir -p gpurun_out/scale
ngpu=$(python -c "import torch; print(torch.cuda.device_count())")
echo "# bench.py scaling sweep ($ngpu GPUs visible)" > $out
echo "" >> $out
echo "| N | bucket MB | NCCL_MIN_NCHANNELS | img/s | ms/step | exposed comm ms | allreduce ms (sum) |" >> $out
echo "|---|---|---|---|---|---|---|" >> $out
row() {   # N bucket chans log
  python - "$@" >> $out <<'PY'
import json, sys
n, b, c, log = sys.argv[1:5]
try:
    r = [json.loads(l) for l in open(log) if l.startswith("{")][-1]
except (IndexError, OSError, ValueError):
    print("| %s | %s | %s | failed | | | |" % (n, b, c)); sys.exit(0)
cm = r.get("comm", {})
print("| %s | %s | %s | %.0f | %.3f | %s | %s |" % (n, b, c, r["value"], r["ms_per_step"],
      cm.get("exposed_comm_ms", ""), cm.get("allreduce_ms_total", "")))
PY
}
port=29600
for n in 1 2 4 8; do
  if [ $n -gt $ngpu ]; then
    echo "| $n | | | skipped: $ngpu GPU(s) on this box | | | |" >> $out
    continue
  fi
  if [ $n -eq 1 ]; then
    log=gpurun_out/scale/n1.log
    timeout -k 10 300 python bench.py --gpus 1 "$@" > $log 2>&1 || exit $?
    row 1 - - $log
    log=gpurun_out/scale/n1_force.log
    MASTER_ADDR=127.0.0.1 MASTER_PORT=$port RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 \
      timeout -k 10 300 python bench.py --gpus 1 --dist_force 1 "$@" > $log 2>&1 || exit $?
    row "1 (RCCL one-rank)" 8 - $log
    continue
  fi
  for b in 2 4 8 16; do
    for ch in unset 16 32; do
      port=$((port + 1))
      log=gpurun_out/scale/n${n}_b${b}_c${ch}.log
      if [ $ch = unset ]; then envc=""; else envc="NCCL_MIN_NCHANNELS=$ch"; fi
      env $envc timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --bucket_mb $b "$@" > $log 2>&1 || exit $?
      row $n $b $ch $log
    done
  done
done
cat $out
