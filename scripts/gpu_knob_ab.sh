set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_db.log 2>&1; tail -2 gpurun_out/t_db.log; grep -E "FAILED" gpurun_out/t_db.log | head -3
UNET_WGRAD_WIN=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_model.py -k "matches_reference or graph" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
bash scripts/gpu_env_sweep.sh UNET_WGRAD_WIN "0 2" 3
for w in 0 2; do UNET_WGRAD_WIN=$w timeout -k 10 200 python tools/layer_times.py --batch 256 --img 128 --out gpurun_out/lt_db_$w.md > /dev/null 2>&1 || exit 1; done
