#!/bin/bash
# Generic same-box A/B of one env knob: selected GPU tests with the knob on, interleaved
# benches, isolated layer times for each value.
#   bash scripts/gpu_knob_ab.sh VAR "v0 v1" "pytest -k expr"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; vals=$2; kexpr=$3
last=${vals##* }
env $var=$last timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "$kexpr" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_knob.log 2>&1; tail -1 gpurun_out/t_knob.log; grep FAILED gpurun_out/t_knob.log | head -3
bash scripts/gpu_env_sweep.sh $var "$vals" 3
for v in $vals; do env $var=$v timeout -k 10 200 python tools/layer_times.py --batch 256 --img 128 --out gpurun_out/lt_knob_$v.md > /dev/null 2>&1 || exit 1; done
