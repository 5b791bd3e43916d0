set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pair.log 2>&1; tail -2 gpurun_out/t_pair.log
bash scripts/gpu_ab.sh --batch 256 --img 128
