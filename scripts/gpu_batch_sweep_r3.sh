#!/bin/bash
# Per-GPU batch sweeps: 3D UNet 128^3 x4 at 2 / 4 / 8 / 16 and the 2D headline at
# 1024 / 2048 (tensors beyond 2 GiB: image-relative buffer offsets).  Writes
# gpurun_out/batch_sweep_r3.md.   bash scripts/gpu_batch_sweep_r3.sh ["3d batches"] ["2d batches"]
set -o pipefail
export TMPDIR=/tmp
b3=${1:-2 4 8 16}; b2=${2:-1024 2048}
mkdir -p gpurun_out/bsweep3
for b in $b3; do
  timeout -k 10 300 python bench.py --dims 3 --img_size 128 --per_gpu_batch $b --steps 6 --warmup 2 \
    > gpurun_out/bsweep3/d3_b$b.log 2>&1 || { tail -5 gpurun_out/bsweep3/d3_b$b.log; exit 1; }
  grep '^{' gpurun_out/bsweep3/d3_b$b.log | cut -c1-200
done
for b in $b2; do
  timeout -k 10 300 python bench.py --per_gpu_batch $b --steps 10 --warmup 3 \
    > gpurun_out/bsweep3/d2_b$b.log 2>&1 || { tail -5 gpurun_out/bsweep3/d2_b$b.log; exit 1; }
  grep '^{' gpurun_out/bsweep3/d2_b$b.log | cut -c1-200
done
python - "$b3" "$b2" <<'PY'
import json, sys
b3, b2 = sys.argv[1].split(), sys.argv[2].split()
out = ["# Per-GPU batch sweeps, round 3 (1x MI355X, bf16, synthetic data)", ""]
for tag, bs, title in (("d3", b3, "3D UNet 128^3 x4 (volumes/sec)"), ("d2", b2, "2D UNet 128x128x4 (images/sec)")):
    out += ["## " + title, "", "| per-GPU batch | value | ms/step | peak device memory (GiB) |", "|---|---|---|---|"]
    for b in bs:
        r = [json.loads(l) for l in open("gpurun_out/bsweep3/%s_b%s.log" % (tag, b)) if l.startswith("{")][0]
        out.append("| %s | %.1f | %.2f | %s |" % (b, r["value"], r["ms_per_step"], r.get("peak_mem_gib")))
    out.append("")
open("gpurun_out/batch_sweep_r3.md", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
