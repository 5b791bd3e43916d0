"""Distributed plumbing on CPU/gloo (BASELINE config #1: world_size=2, 64x64 synthetic):
gradient averaging, replica consistency, rank-0-only side effects, launcher and
fail-fast behaviour, checkpoint resume."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.grad_sync import GradSync, plan_buckets
    from unet_distributed_amd.runtime.backends import TorchBackend
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.params import FlatParams
    ctx = D.init("cpu", "gloo", 60)
    cfg = Config(batch_size=4, img_size=32, dtype="fp32", in_channels=4, dropout=0.0)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=rank))      # different inits...
    D.broadcast_(flat.master, 0)                                  # ...made identical by broadcast
    be = TorchBackend(spec, flat, cfg, "cpu", 2)
    bounds = plan_buckets(flat, 0.5)
    sync = GradSync(flat, bounds, ctx, overlap=True)
    x, y = synthetic_brats(2, 32, 4, seed=100 + rank)
    be.fwd_bwd(torch.from_numpy(x), torch.from_numpy(y), seed=1)
    local = flat.grad.clone()
    allg = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    for i in range(len(bounds)):
        sync.on_segment(i)
    sync.finish()
    mean = torch.stack(allg).mean(0)
    ok_avg = torch.allclose(flat.grad, mean, atol=1e-6)
    opt = TFAdam(flat, cfg)
    opt.step()
    s = flat.master.double().sum().reshape(1)
    mx, mn = s.clone(), s.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    res = dict(rank=rank, ok_avg=bool(ok_avg), same=bool((mx - mn).abs().item() == 0.0), nbuckets=len(bounds))
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    D.destroy()


def test_gloo_bucketed_allreduce_equals_mean_and_replicas_agree(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = json.load(open(tmp_path / ("r%d.json" % r)))
        assert res["ok_avg"] and res["same"] and res["nbuckets"] > 1


def _run_train(tmp_path, extra, nproc=2, timeout=600):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "train.py"),
           "--synthetic", "--device", "cpu", "--dtype", "fp32", "--img_size", "64", "--in_channels", "4",
           "--batch_size", "4", "--synthetic_train", "8", "--synthetic_test", "4", "--log_every", "1",
           "--checkpoint_dir", str(tmp_path / "ck"), "--log_jsonl", str(tmp_path / "m.jsonl")] + extra
    return subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=timeout)


@pytest.mark.slow
def test_train_py_two_ranks_gloo_end_to_end_and_resume(tmp_path):
    r = _run_train(tmp_path, ["--epochs", "1"])
    assert r.returncode == 0, r.stdout[-3000:]
    assert "TEST DATASET" in r.stdout and "Finished work on this node." in r.stdout
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert [x["step"] for x in recs if x["kind"] == "train"] == [1, 2]      # rank 0 only logs
    logdir = tmp_path / "ck" / "unet,lr=0.0005,conv2DTranspose,intra=50,inter=2"
    assert (logdir / "checkpoint").exists() and (tmp_path / "ck" / "last_good_model.cpkt.index").exists()
    assert (tmp_path / "ck" / "saved_model" / "saved_model.json").exists()
    # resume: 2 epochs total -> continues from global_step 2
    r2 = _run_train(tmp_path, ["--epochs", "2"])
    assert r2.returncode == 0, r2.stdout[-3000:]
    assert "Restored checkpoint at global_step 2" in r2.stdout
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert [x["step"] for x in recs if x["kind"] == "train"][-2:] == [3, 4]


@pytest.mark.slow
def test_rank_failure_fails_fast(tmp_path):
    r = _run_train(tmp_path, ["--epochs", "3", "--fault_inject_step", "1", "--fault_inject_rank", "1",
                              "--dist_timeout_s", "60", "--no_checkpoint"], timeout=300)
    assert r.returncode != 0
    assert "fault injected" in r.stdout


def test_parameter_server_applies_tf_adam_in_arrival_order():
    sys.path.insert(0, ROOT)
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel.async_ps import ParameterServer
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.params import FlatParams
    cfg = Config(img_size=32, in_channels=1, const_learningrate=False, decay_steps=3)
    spec = spec_from_config(cfg)
    a, b = FlatParams(spec), FlatParams(spec)
    a.load_dict(reference.init_params(spec, seed=0))
    b.master.copy_(a.master)
    ps = ParameterServer(a, cfg)
    opt = TFAdam(b, cfg)
    out = torch.zeros_like(a.master)
    g = torch.Generator().manual_seed(0)
    for k in range(4):                         # four "workers'" gradients in arrival order
        grad = torch.randn(a.numel, generator=g)
        step = ps.apply(grad, out)
        b.grad.copy_(grad)
        opt.step()
        assert step == b.global_step == k + 1
    assert torch.allclose(out, b.master, atol=1e-7)
    assert abs(ps.b1p - b.beta1_power) < 1e-12


@pytest.mark.slow
def test_async_ps_mode_two_ranks(tmp_path):
    r = _run_train(tmp_path, ["--is_sync", "0", "--steps", "6", "--no_checkpoint"])
    assert r.returncode == 0, r.stdout[-3000:]
    assert "Worker #1 reports job finished." in r.stdout
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    steps = [x["step"] for x in recs if x["kind"] == "train"]
    assert len(steps) == 3 and steps[-1] <= 6           # 3 local steps; PS global_step advances per worker step
    assert [x["step"] for x in recs if x["kind"] == "test_final"] == [6]   # PS global_step at the end


@pytest.mark.slow
def test_async_ps_fp16_overflow_on_one_rank_keeps_ranks_in_lockstep(tmp_path):
    """An fp16 overflow on rank 1 at its very first step (the most likely overflow,
    at the 2^16 initial scale) must not desynchronise the per-epoch evaluations: a
    skipped iteration that did not count would leave that rank at local step 0, a
    multiple of the epoch length, and send it into evaluate()'s allreduce alone."""
    r = _run_train(tmp_path, ["--is_sync", "0", "--epochs", "2", "--dtype", "fp16", "--no_checkpoint",
                              "--fault_inject_overflow_step", "0", "--fault_inject_rank", "1",
                              "--dist_timeout_s", "60"], timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len([x for x in recs if x["kind"] == "test"]) >= 1
    assert len([x for x in recs if x["kind"] == "test_final"]) == 1


@pytest.mark.slow
def test_sync_fp16_overflow_on_one_rank_skips_the_step_on_every_rank(tmp_path):
    """Sync mode (the default): rank 1's gradient overflows at step 0.  The poison is
    written before the allreduce of the bucket that holds it, so BOTH ranks see the
    non-finite average and skip that step together; it fires once (the retried step
    carries the same number), the replicas stay identical (checked every step) and
    training reaches its final step."""
    r = _run_train(tmp_path, ["--epochs", "2", "--dtype", "fp16", "--no_checkpoint",
                              "--fault_inject_overflow_step", "0", "--fault_inject_rank", "1",
                              "--check_sync_every", "1", "--dist_timeout_s", "60"], timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    train = [x for x in recs if x["kind"] == "train"]
    assert train and train[-1]["step"] == 4                 # 2 epochs x 2 global batches
    assert [x["step"] for x in recs if x["kind"] == "test_final"] == [4]


def _run_launcher(tmp_path, extra, timeout=600):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "launch.py"), "--nproc_per_node", "2", "--master_port", str(port),
           "--log_dir", str(tmp_path / "logs"), "--grace_s", "5", "--", os.path.join(ROOT, "train.py"),
           "--synthetic", "--device", "cpu", "--dtype", "fp32", "--img_size", "32", "--in_channels", "4",
           "--batch_size", "4", "--synthetic_train", "8", "--synthetic_test", "4",
           "--checkpoint_dir", str(tmp_path / "ck"), "--no_checkpoint"] + extra
    return subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=timeout)


@pytest.mark.slow
def test_launcher_runs_ranks_and_stops_node_on_failure(tmp_path):
    r = _run_launcher(tmp_path, ["--steps", "2"])
    assert r.returncode == 0, r.stdout[-3000:]
    log0 = open(tmp_path / "logs" / "training.rank0.log").read()
    assert "Finished work on this node." in log0
    assert os.path.exists(tmp_path / "logs" / "training.rank1.log")
    # rank 1 dies at step 1 while rank 0 would block in the allreduce: the launcher
    # must tear rank 0 down long before the 600 s collective timeout
    import time
    t0 = time.time()
    r = _run_launcher(tmp_path, ["--steps", "50", "--fault_inject_step", "1", "--fault_inject_rank", "1"])
    assert r.returncode != 0
    assert time.time() - t0 < 120
    assert "rank 1 exited" in r.stdout


def test_inventory_roundtrip_and_remote_commands(tmp_path):
    sys.path.insert(0, ROOT)
    from unet_distributed_amd import launch
    p = str(tmp_path / "inv.yml")
    launch.write_inventory(p, ["10.0.0.1", "10.0.0.2"])
    hosts = launch.read_inventory(p)
    assert hosts == ["10.0.0.1", "10.0.0.2"]
    cmds = launch.remote_commands(hosts, "/w", 8, 29500, ["train.py", "--epochs", "2"])
    assert len(cmds) == 2 and "--node_rank 1" in cmds[1][-1] and "--master_addr 10.0.0.1" in cmds[1][-1]
    env = launch.child_env({}, 9, 1, 16, 8, "10.0.0.1", 29500)
    assert env["RANK"] == "9" and env["LOCAL_RANK"] == "1" and env["WORLD_SIZE"] == "16"


def _run_bench(extra, nproc=2, timeout=600, env_extra=None):
    """The driver's multi-GPU bench command (`torch.distributed.run ... bench.py --gpus N`)."""
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc)] + extra
    return subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=timeout, cwd=ROOT)


def bench_record(out):
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(recs) == 1, out[-3000:]          # rank 0 prints exactly one JSON line
    return recs[0]


def check_multirank_bench(rec, n):
    """The fields the driver and the judge read from an N-rank bench line, plus the
    per-bucket / exposed-communication diagnostics of the N > 1 branch."""
    assert rec["n_gpus"] == n and rec["config"]["parallelism"] == "dp%d" % n
    assert rec["config"]["global_batch"] == n * rec["config"]["per_gpu_batch"]
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["scaling"] == "weak"
    c = rec["comm"]
    assert c["world_size"] == n
    per = c["allreduce_ms_per_bucket"]
    assert len(per) == len(c["buckets_mb"]) >= 2 and all(t > 0 for t in per)
    for k in ("exposed_comm_ms", "step_ms_serial_comm", "step_ms_overlapped", "step_ms_compute_only"):
        assert isinstance(c[k], float), (k, c)


def test_bench_py_two_ranks_gloo_cpu():
    """bench.py's N > 1 code path (timed steps with overlapped bucket allreduces, MAX over
    ranks, then comm_diagnostics: per-bucket allreduce times and the overlapped / serial /
    compute-only A/B) on two CPU ranks over gloo with the ATen backend -- the same command
    shape the driver's 8-GPU lease runs (`test_dist.py:385-398`: every worker's sharded step)."""
    r = _run_bench(["--backend", "torch", "--dtype", "fp32", "--per_gpu_batch", "2", "--img_size", "64",
                    "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stdout[-3000:]
    rec = bench_record(r.stdout)
    check_multirank_bench(rec, 2)
    assert rec["comm"]["backend"] == "gloo" and rec["config"]["backend"] == "torch"


@pytest.mark.slow
def test_bench_py_eight_ranks_gloo_cpu():
    """Rehearsal of the driver's 8-GPU lease command shape (`torch.distributed.run
    --nproc-per-node 8 bench.py --gpus 8`) at world 8 on CPU/gloo: rank 0 prints one
    line with n_gpus / global_batch / parallelism of the 8-rank job, every bucket gets an
    allreduce time and the exposed-communication A/B is reported (`test_dist.py:385-398`)."""
    r = _run_bench(["--backend", "torch", "--dtype", "fp32", "--per_gpu_batch", "1", "--img_size", "32",
                    "--steps", "2", "--warmup", "1", "--bucket_mb", "4"], nproc=8,
                   env_extra={"OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stdout[-3000:]
    rec = bench_record(r.stdout)
    check_multirank_bench(rec, 8)
    assert rec["config"]["global_batch"] == 8 and rec["comm"]["backend"] == "gloo"
    assert len(rec["comm"]["buckets_mb"]) >= 4          # 29.6 MiB of fp32 gradients in 4 MiB buckets


@pytest.mark.slow
def test_train_py_four_ranks_kill_and_resume(tmp_path):
    """SURVEY §4 tier 5 at world 4: a rank dies mid-run (the job fails fast, nothing
    hangs), the relaunched job restores the last periodic checkpoint written before the
    fault and trains only the remaining steps (`test_dist.py:347-362,380-381`)."""
    extra = ["--steps", "6", "--save_model_secs", "0", "--dist_timeout_s", "60"]
    r = _run_train(tmp_path, extra + ["--fault_inject_step", "3", "--fault_inject_rank", "2"], nproc=4,
                   timeout=300)
    assert r.returncode != 0 and "fault injected at step 3 on rank 2" in r.stdout, r.stdout[-3000:]
    logdir = tmp_path / "ck" / "unet,lr=0.0005,conv2DTranspose,intra=50,inter=2"
    assert "model_checkpoint_path: \"model.ckpt-3\"" in (logdir / "checkpoint").read_text()
    r2 = _run_train(tmp_path, extra, nproc=4, timeout=300)
    assert r2.returncode == 0, r2.stdout[-3000:]
    assert "Restored checkpoint at global_step 3" in r2.stdout
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    steps = [x["step"] for x in recs if x["kind"] == "train"]
    assert steps[:3] == [1, 2, 3] and steps[3:] == [4, 5, 6]
    assert [x["step"] for x in recs if x["kind"] == "test_final"] == [6]
