#!/bin/bash
# Same-box A/B of an env knob on bench.py (interleaved rounds): bash scripts/gpu_ab_env.sh VAR A B [rounds] [bench args]
set -o pipefail
export TMPDIR=/tmp
var=$1; a=$2; b=$3; rounds=${4:-3}; shift 4 || shift $#
mkdir -p gpurun_out/ab
for r in $(seq 1 $rounds); do
  for v in $a $b; do
    env $var=$v timeout -k 10 200 python bench.py "$@" > gpurun_out/ab/${var}_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('$var=$v round $r', r['value'], r['ms_per_step'])" gpurun_out/ab/${var}_${v}_$r.log
  done
done
