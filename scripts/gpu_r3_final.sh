#!/bin/bash
# Round-3 end evidence: headline profile (kernel stats, per-launch times, PMC table),
# one-step timelines (headline / BN / GN fp16) and the side-config benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_profile.sh r3end > gpurun_out/prof_r3end.log 2>&1 || { echo "profile rc=$?"; exit 1; }
echo profile done
bash scripts/gpu_timeline.sh r3end > gpurun_out/tl_r3end.log 2>&1 || { echo "timeline rc=$?"; exit 1; }
echo timeline done
bash scripts/gpu_configs.sh
