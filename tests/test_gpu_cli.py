"""The training CLI on the GPU: one GPU path.  The reference's own precision (fp32,
`test_dist.py:196-202`) runs on the native fp32 executor (runtime/f32_engine.py); a config
no HIP executor takes (fp32 with BatchNorm) must exit non-zero and name the reason instead
of silently running ATen / MIOpen; the same config runs when the ATen path is asked for
explicitly (--backend torch)."""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(tmp_path, extra):
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--synthetic", "--img_size", "64", "--in_channels", "4",
           "--batch_size", "4", "--synthetic_train", "8", "--synthetic_test", "4", "--epochs", "1",
           "--no_checkpoint", "--log_jsonl", str(tmp_path / "m.jsonl")] + extra
    return subprocess.run(cmd, env=dict(os.environ, PYTHONPATH=ROOT), stdout=subprocess.PIPE,
                          stderr=subprocess.STDOUT, text=True, timeout=240, cwd=ROOT)


def test_train_fp32_on_gpu_runs_native(cuda_dev, tmp_path):
    r = _train(tmp_path, ["--dtype", "fp32"])
    assert r.returncode == 0, r.stdout[-3000:]
    assert "backend native" in r.stdout, r.stdout[-2000:]


def test_train_fp32_batchnorm_on_gpu_fails_loudly(cuda_dev, tmp_path):
    r = _train(tmp_path, ["--dtype", "fp32", "--norm", "batch"])
    assert r.returncode != 0, r.stdout[-2000:]
    assert "native HIP executor does not support" in r.stdout and "norm=batch" in r.stdout, r.stdout[-2000:]


def test_train_bf16_on_gpu_runs_native(cuda_dev, tmp_path):
    r = _train(tmp_path, ["--dtype", "bf16"])
    assert r.returncode == 0, r.stdout[-3000:]
    assert "backend native" in r.stdout, r.stdout[-2000:]
