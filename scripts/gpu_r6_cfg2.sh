#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
SKIP_MAIN=1 SKIP_FP32=1 bash scripts/gpu_r6_configs.sh "" "" || exit 1
