#!/bin/bash
# Build a baseline copy of the package at git revision $1 (default HEAD) into ab_base/
# so one GPU call can A/B the working tree against it on the same box:
#   bash scripts/ab_base.sh HEAD
#   gpurun -- 'python tools/layer_times.py --out gpurun_out/lt_new.md &&
#              (cd ab_base && python tools/layer_times.py --out ../gpurun_out/lt_base.md)'
set -e
rev=${1:-HEAD}
root=$(git rev-parse --show-toplevel)
rm -rf "$root/ab_base" /tmp/ab_wt
git -C "$root" worktree prune
git -C "$root" worktree add --detach /tmp/ab_wt "$rev" > /dev/null
(cd /tmp/ab_wt && python -m unet_distributed_amd.native.build > /dev/null)
mkdir -p "$root/ab_base"
cp -r /tmp/ab_wt/unet_distributed_amd /tmp/ab_wt/tools /tmp/ab_wt/bench.py "$root/ab_base/"
find "$root/ab_base" -name "*.o" -delete
rm -rf "$root/ab_base/unet_distributed_amd/csrc"
git -C "$root" worktree remove --force /tmp/ab_wt
echo "ab_base/ = $(git -C "$root" rev-parse --short "$rev")"
