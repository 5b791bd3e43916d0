#!/bin/bash
# Bucket-size x channel sweep of the multi-GPU headline on ONE 8-GPU node (first lease):
# bucket_mb 2/4/8/16/32 x NCCL_MIN_NCHANNELS default/8/16, each a full bench.py run
# (timed steps + comm diagnostics: per-bucket allreduce ms, exposed / serial comm).
# Results: gpurun_out/sweep/<bucket>_<ch>.json ; summary table on stdout.
#   bash scripts/gpu_bucket_sweep.sh [ngpus]
set -o pipefail
export TMPDIR=/tmp
N=${1:-8}
mkdir -p gpurun_out/sweep
port=29600
for ch in default 8 16; do
  for mb in 2 4 8 16 32; do
    port=$((port + 1))
    env_ch=""
    [ "$ch" != default ] && env_ch="NCCL_MIN_NCHANNELS=$ch"
    env $env_ch timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --steps 20 --warmup 5 --bucket_mb $mb \
      > gpurun_out/sweep/${mb}_${ch}.log 2>&1 || { echo "bucket $mb ch $ch failed"; tail -5 gpurun_out/sweep/${mb}_${ch}.log; exit 1; }
    grep '^{' gpurun_out/sweep/${mb}_${ch}.log > gpurun_out/sweep/${mb}_${ch}.json
  done
done
python - <<'PY'
import glob, json, os
rows = []
for f in sorted(glob.glob("gpurun_out/sweep/*.json")):
    r = json.loads(open(f).read().splitlines()[0]); c = r.get("comm", {})
    rows.append((os.path.basename(f)[:-5], r["value"], r["ms_per_step"], c.get("allreduce_ms_total"),
                 c.get("exposed_comm_ms"), c.get("serial_comm_ms"), c.get("buckets_mb")))
print("| bucket_ch | img/s | ms/step | allreduce ms | exposed ms | serial ms | buckets MB |")
print("|---|---|---|---|---|---|---|")
for r in rows:
    print("| %s | %s | %s | %s | %s | %s | %s |" % r)
PY
