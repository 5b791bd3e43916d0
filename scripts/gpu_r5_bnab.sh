#!/bin/bash
# Same-box A/B of the per-column-block BatchNorm finalize + norm-pass grid (this tree) against
# the tree before it (ab_old = 7829196): BatchNorm and GroupNorm fp16 benches, interleaved.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_ab_tree.sh ab_old 3 --norm batch --steps 10 --warmup 3 || exit 1
mv gpurun_out/abt gpurun_out/abt_bn
bash scripts/gpu_ab_tree.sh ab_old 2 --norm group --dtype fp16 --steps 10 --warmup 3 || exit 1
mv gpurun_out/abt gpurun_out/abt_gn
