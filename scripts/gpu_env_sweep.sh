#!/bin/bash
# Interleaved bench sweep of one environment knob on the same box:
#   bash scripts/gpu_env_sweep.sh VAR "v1 v2 ..." [rounds] [bench args...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; vals=$2; rounds=${3:-2}; shift 3
for r in $(seq 1 $rounds); do
  for v in $vals; do
    line=$(env $var=$v timeout -k 10 180 python bench.py "$@" 2>/dev/null | grep metric) || exit $?
    echo "$var=$v round=$r $(echo $line | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done | tee gpurun_out/env_sweep_$var.txt
