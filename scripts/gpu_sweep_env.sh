#!/bin/bash
# Same-box sweep of an env knob on bench.py (interleaved rounds):
#   bash scripts/gpu_sweep_env.sh VAR "v1 v2 ..." [rounds] [bench args]
set -o pipefail
export TMPDIR=/tmp
var=$1; vals=$2; rounds=${3:-2}; shift 3 || shift $#
mkdir -p gpurun_out/sweep
for r in $(seq 1 $rounds); do
  for v in $vals; do
    env $var=$v timeout -k 10 200 python bench.py "$@" > gpurun_out/sweep/${var}_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('$var=$v round $r', r['value'], r['ms_per_step'])" gpurun_out/sweep/${var}_${v}_$r.log
  done
done
