#!/bin/bash
# Same-box A/B of two source trees (interleaved rounds): the current tree against an
# exported older tree with its own built extension (e.g. `git archive <rev> | tar -x -C ab_old`
# + `python -m unet_distributed_amd.native.build` inside it).
#   bash scripts/gpu_ab_tree.sh <old_tree_dir> [rounds] [bench args]
set -o pipefail
export TMPDIR=/tmp
old=$1; rounds=${2:-3}; shift 2 || shift $#
mkdir -p gpurun_out/abt
for r in $(seq 1 $rounds); do
  for t in old new; do
    if [ $t = old ]; then d=$old; else d=.; fi
    (cd $d && timeout -k 10 200 python bench.py "$@") > gpurun_out/abt/${t}_$r.log 2>&1 || exit $?
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('$t round $r', r['value'], r['ms_per_step'])" gpurun_out/abt/${t}_$r.log
  done
done
