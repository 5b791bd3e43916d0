set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "upsample or matches_reference or chunked" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
bash scripts/gpu_env_sweep.sh UNET_UPS_MATERIALIZE "0 1" 2 --use_upsampling --in_channels 1 --steps 10 --warmup 3
