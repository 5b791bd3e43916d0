#!/bin/bash
# train.py steady-state throughput vs bench.py on the same box (headline config:
# 128x128x4 bf16, per-GPU batch 256, HBM-resident synthetic data).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/train_speed.jsonl
timeout -k 10 400 python train.py --synthetic --in_channels 4 --batch_size 256 --synthetic_train 7680 \
  --synthetic_test 256 --epochs 1 --log_every 5 --no_checkpoint --noexport --noprogress \
  --log_jsonl gpurun_out/train_speed.jsonl > gpurun_out/train_speed.log 2>&1 || { tail -20 gpurun_out/train_speed.log; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_speed.log 2>&1 || exit $?
python - <<'PY'
import json, statistics
recs = [json.loads(l) for l in open("gpurun_out/train_speed.jsonl") if l.strip()]
ips = [r["images_per_sec"] for r in recs if r.get("kind") == "train" and "images_per_sec" in r]
b = [json.loads(l) for l in open("gpurun_out/bench_speed.log") if l.startswith("{")][0]
steady = statistics.median(ips[1:])
print("train.py img/s per log window:", [round(v) for v in ips])
print("train.py steady (median, first window dropped): %.0f  bench.py: %.0f  ratio %.3f" % (steady, b["value"], steady / b["value"]))
PY
