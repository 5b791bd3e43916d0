#!/bin/bash
# Same-box interleaved sweep of executor tunables on the headline bench (UNET_ENGINE values).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
for r in 1 2; do
  for v in "$@"; do
    UNET_ENGINE=$v timeout -k 10 200 python bench.py > gpurun_out/sw/run.log 2>&1 || exit 1
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('$v round $r', r['value'], r['ms_per_step'])" gpurun_out/sw/run.log
  done
done
