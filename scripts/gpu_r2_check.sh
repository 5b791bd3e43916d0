set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1 || { tail -40 gpurun_out/pytest_r2b.log; exit 1; }
tail -3 gpurun_out/pytest_r2b.log
bash scripts/gpu_trainer_speed.sh
