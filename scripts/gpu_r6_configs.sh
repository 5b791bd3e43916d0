#!/bin/bash
# Round 6: every BASELINE config at N=1 on the current tree (+ per-GPU batch sweeps of
# 512^2 and 3D), TF/s beside img/s -> gpurun_out/r6_configs.jsonl / r6_configs.md.
#   bash scripts/gpu_r6_configs.sh ["512 batches"] ["3d batches"]
set -o pipefail
export TMPDIR=/tmp
b512=${1-16 32 64 128}; b3=${2-8 12 16}
o=gpurun_out/r6cfg; mkdir -p $o; : > $o/configs.jsonl
run() { tag=$1; shift
  timeout -k 10 600 python bench.py "$@" > $o/$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -20 $o/$tag.log; exit 1; }
  python - "$tag" "$o/$tag.log" "$*" >> $o/configs.jsonl <<'PY'
import json, sys
sys.path.insert(0, "tools")
from config_flops import step_flops_per_image as f
tag, log, args = sys.argv[1], sys.argv[2], sys.argv[3].split()
r = [json.loads(l) for l in open(log) if l.startswith("{")][0]
g = lambda k, d: type(d)(args[args.index(k) + 1]) if k in args else d
fl = f(g("--img_size", 128), g("--in_channels", 4), g("--dims", 2), "--use_upsampling" in args)
r["tag"], r["args"] = tag, " ".join(args)
r["gflop_per_img"] = round(fl / 1e9, 3)
r["tflops"] = round(r["value"] * fl / 1e12, 1)
print(json.dumps(r))
PY
  tail -1 $o/configs.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], d['value'], d['ms_per_step'], d['tflops'], 'TF/s', d.get('train_dice_last_batch'))"
}
[ -n "$SKIP_MAIN" ] || { run headline --steps 20 --warmup 5
run bn --norm batch --steps 10 --warmup 3
run gn16 --norm group --dtype fp16 --steps 10 --warmup 3
run ups --use_upsampling --in_channels 1 --steps 10 --warmup 3; }
for b in $b512; do run s512_b$b --img_size 512 --in_channels 1 --per_gpu_batch $b --steps 8 --warmup 3; done
for b in $b3; do run d3_b$b --dims 3 --per_gpu_batch $b --steps 5 --warmup 2; done
[ -n "$SKIP_FP32" ] || { run fp32_native --dtype fp32 --per_gpu_batch 128 --steps 5 --warmup 2
export MIOPEN_FIND_MODE=NORMAL   # (FAST picks naive fp32 NHWC kernels: profiles/r5_aten_ups_kernels.md)
run fp32_aten --dtype fp32 --backend torch --per_gpu_batch 128 --steps 5 --warmup 2; }
run fp32_native_b512 --dtype fp32 --per_gpu_batch 512 --steps 5 --warmup 2
# the bucketed RCCL path at one rank (process group + per-bucket collectives in the timed step)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --dist_force 1 --steps 10 --warmup 3 > $o/dist_force.log 2>&1 || { echo "dist_force rc=$?"; tail -20 $o/dist_force.log; exit 1; }
grep '^{' $o/dist_force.log
