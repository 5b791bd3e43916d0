#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/dbg_dw_det.py 2>&1 | grep -v amdgpu.ids | tail -20
