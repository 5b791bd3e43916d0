#!/bin/bash
# Executor option sweep on the BatchNorm step (defaults were tuned on the headline):
# 2 interleaved same-box reps per setting.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bnsweep
for r in 1 2; do
  for o in default wg_target=384 wg_target=768 win_pf=16 win_cp=0 dw_wgs=1024 dual_stream=0; do
    if [ $o = default ]; then e=""; else e=$o; fi
    UNET_ENGINE=$e timeout -k 10 200 python bench.py --norm batch --steps 10 --warmup 3 > gpurun_out/bnsweep/${o}_$r.log 2>&1 || exit $?
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('$o rep $r', r['value'], r['ms_per_step'])" gpurun_out/bnsweep/${o}_$r.log
  done
done
