#!/bin/bash
# Per-launch layer times under two values of an env knob: bash scripts/gpu_lt_ab.sh VAR A B
export TMPDIR=/tmp
var=$1; a=$2; b=$3
mkdir -p gpurun_out/lt
for v in $a $b; do
  env $var=$v timeout -k 10 300 python tools/layer_times.py --batch ${BATCH:-1024} --img 128 \
    --out gpurun_out/lt/${var}_$v.md > gpurun_out/lt/${var}_$v.log 2>&1 || exit $?
done
