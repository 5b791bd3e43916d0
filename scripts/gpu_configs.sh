#!/bin/bash
# Benchmarks of the BASELINE.json side configs on one MI355X (each under its own limit).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/configs.log; : > $o
run() { timeout -k 10 240 python bench.py "$@" 2>/dev/null | grep metric >> $o || { echo "FAILED: $*" >> $o; exit 1; }; }
run --steps 20 --warmup 5
run --steps 20 --warmup 5 --per_gpu_batch 256
run --dims 3 --steps 6 --warmup 2
run --img_size 512 --in_channels 1 --per_gpu_batch 16 --steps 10 --warmup 3
run --dtype fp16 --norm group --per_gpu_batch 1024 --steps 10 --warmup 3
run --norm batch --steps 10 --warmup 3
run --use_upsampling --in_channels 1 --steps 10 --warmup 3
python - <<'PY'
import json
for l in open("gpurun_out/configs.log"):
    if l.startswith("FAILED"): print(l.strip()); continue
    d = json.loads(l)
    c = d["config"]
    print("%-60s %10.1f %s  %.2f ms/step  batch %d" % (c["model"][:60], d["value"], d["unit"], d["ms_per_step"], c["per_gpu_batch"]))
PY
