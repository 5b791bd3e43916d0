"""The RCCL (``nccl`` backend) code paths on real GPUs.

* One rank (runs on the 1-GPU box): ``dist.init(force=True)`` builds a one-rank RCCL
  communicator, so the nccl-only lines -- ``device_id`` binding, ``barrier(device_ids)``,
  ``ReduceOp.AVG`` buckets issued from the executor's side stream between backward
  segments, ``work.wait()`` ordering the caller's stream -- run for real.  Ordering is
  checked by poisoning the gradient buffer with NaN before every step: an allreduce
  that ran before its segment's kernels (or a reader that ran before the allreduce's
  in-place write-back) leaves NaN / stale values behind.
* ``bench.py --dist_force 1`` times the step WITH the one-rank bucket allreduces and
  reports the per-bucket RCCL time (comm diagnostics).
* The DeviceParameterServer (one native TF-Adam launch per push) against the CPU
  reference ParameterServer over several pushes.
* Two ranks on two GPUs (skipped on a 1-GPU box, run unchanged on the first multi-GPU
  lease): the bucket average over RCCL, and the async parameter server with its RCCL
  data plane through an epoch boundary (evaluation collectives beside the server
  thread's point-to-point traffic).
Reference: `test_dist.py:130-131` (cluster / server), `test_dist.py:249-267` (sync /
async updates)."""

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ngpu():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def _env(rank, world, port, local):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(local))
    os.environ.pop("UNET_DIST_BACKEND", None)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.path.insert(0, ROOT)


def _entries_equal(flat, a, b):
    return all(torch.equal(a[off:off + n], b[off:off + n]) for _, _, off, n in flat.entries)


def _world1(rank, port, out):
    _env(0, 1, port, 0)
    import torch.distributed as dist
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.grad_sync import GradSync, plan_buckets
    from unet_distributed_amd.runtime.backends import NativeBackend
    from unet_distributed_amd.runtime.params import FlatParams
    ctx = D.init("cuda", "nccl", 120, force=True)
    rec = dict(backend=ctx.backend, pg_world=dist.get_world_size(), initialized=ctx.initialized)
    D.barrier()                                             # barrier(device_ids=[...]) on RCCL
    dev = ctx.device
    cfg = Config(batch_size=4, img_size=64, in_channels=4, hip_graph=True)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=3))
    bounds = plan_buckets(flat, 0.25)
    be = NativeBackend(spec, flat, cfg, dev, 4, bounds)
    be.engine.repack()
    x, y = synthetic_brats(4, 64, 4, seed=9)
    x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    nan = float("nan")
    flat.grad.fill_(nan)
    be.fwd_bwd(x, y, seed=5)
    torch.cuda.synchronize()
    ref = flat.grad.clone()
    ok = {}
    for name, overlap in (("overlap", True), ("serial", False)):
        sync = GradSync(flat, bounds, ctx, overlap=overlap, force=True)
        assert sync.active and sync.avg_native
        good = True
        for rep in range(3):
            flat.grad.fill_(nan)
            be.fwd_bwd(x, y, seed=5, on_segment=sync.on_segment)
            sync.finish()
            snap = flat.grad.clone()                        # first reader on the caller's stream
            torch.cuda.synchronize()
            good = good and _entries_equal(flat, snap, ref) and _entries_equal(flat, flat.grad, ref)
        ok[name] = bool(good)
    finite = all(bool(torch.isfinite(ref[off:off + n]).all().item()) for _, _, off, n in flat.entries)
    rec.update(ok=ok, buckets=len(bounds), finite=finite)
    with open(os.path.join(out, "w1.json"), "w") as f:
        json.dump(rec, f)
    D.destroy()


def test_rccl_one_rank_bucket_path_orders_streams(tmp_path):
    """nccl at WORLD_SIZE=1: device-bound init, device barrier, AVG buckets from the side
    stream; the gradients equal the no-communication step bit for bit, every time, with
    the buffer NaN-poisoned before each step (ordering of segment -> allreduce ->
    caller's stream)."""
    mp.spawn(_world1, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    r = json.load(open(tmp_path / "w1.json"))
    assert r["backend"] == "nccl" and r["pg_world"] == 1 and r["initialized"]
    assert r["buckets"] >= 3 and r["finite"]
    assert r["ok"] == {"overlap": True, "serial": True}, r


def test_bench_dist_force_one_rank_reports_rccl_buckets():
    """bench.py --dist_force 1 at one rank: the timed step includes the RCCL bucket
    allreduces and the JSON carries the comm diagnostics (per-bucket RCCL time)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.pop("UNET_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist_force", "1", "--per_gpu_batch", "64",
                        "--steps", "3", "--warmup", "2"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    c = rec["comm"]
    assert c["backend"] == "nccl" and c["world_size"] == 1
    assert len(c["allreduce_ms_per_bucket"]) == len(c["buckets_mb"]) >= 3
    assert all(t > 0 for t in c["allreduce_ms_per_bucket"])
    assert c["step_ms_overlapped"] > 0 and rec["value"] > 0


def test_device_parameter_server_matches_cpu_reference(cuda_dev):
    """The GPU-resident PS (one fused native TF-Adam launch per push, server stream)
    against the CPU ParameterServer: weights, both Adam slots and the step after
    several pushes with decaying LR (fp32 TF-Adam on both sides)."""
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel.async_ps import DeviceParameterServer, ParameterServer
    from unet_distributed_amd.runtime.params import FlatParams
    cfg = Config(img_size=64, in_channels=4, const_learningrate=False, decay_steps=2, learning_rate=1e-3)
    spec = spec_from_config(cfg)
    fd, fc = FlatParams(spec, device=cuda_dev), FlatParams(spec)
    init = reference.init_params(spec, seed=4)
    fd.load_dict(init)
    fc.load_dict(init)
    dps, cps = DeviceParameterServer(fd, cfg), ParameterServer(fc, cfg)
    od, oc = torch.zeros_like(fd.master), torch.zeros_like(fc.master)
    g = torch.Generator().manual_seed(1)
    for k in range(5):
        grad = torch.randn(fc.numel, generator=g) * 1e-2
        sd = dps.apply(grad.to(cuda_dev), od)
        sc = cps.apply(grad, oc)
        assert sd == sc == k + 1
    dps.stream.synchronize()
    tol = dict(rtol=1e-5, atol=1e-7)
    assert torch.allclose(od.cpu(), oc, **tol)
    assert torch.allclose(dps.w.cpu(), cps.w, **tol)
    assert torch.allclose(dps.m.cpu(), cps.m, **tol) and torch.allclose(dps.v.cpu(), cps.v, **tol)
    assert abs(dps.b1p - cps.b1p) < 1e-12 and abs(dps.b2p - cps.b2p) < 1e-12


def _two(rank, world, port, out):
    _env(rank, world, port, rank)
    import torch.distributed as dist
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.grad_sync import GradSync, plan_buckets
    from unet_distributed_amd.runtime.backends import NativeBackend
    from unet_distributed_amd.runtime.params import FlatParams
    ctx = D.init("cuda", "auto", 120)
    dev = ctx.device
    cfg = Config(batch_size=4 * world, img_size=64, in_channels=4, hip_graph=True)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=7 + rank))
    D.broadcast_(flat.master, 0)
    bounds = plan_buckets(flat, 0.25)
    be = NativeBackend(spec, flat, cfg, dev, 4, bounds)
    be.engine.repack()
    x, y = synthetic_brats(4, 64, 4, seed=100 + rank)
    x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    be.fwd_bwd(x, y, seed=5 + rank)
    torch.cuda.synchronize()
    local = flat.grad.detach().clone()
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    mean = torch.stack(gathered).mean(0)
    sync = GradSync(flat, bounds, ctx, overlap=True)
    be.fwd_bwd(x, y, seed=5 + rank, on_segment=sync.on_segment)
    sync.finish()
    torch.cuda.synchronize()
    rec = dict(rank=rank, backend=ctx.backend, max_err=(flat.grad - mean).abs().max().item(),
               scale=mean.abs().max().item(), local_diff=(local - mean).abs().max().item())
    with open(os.path.join(out, "t%d.json" % rank), "w") as f:
        json.dump(rec, f)
    D.destroy()


@pytest.mark.skipif(_ngpu() < 2, reason="needs two GPUs (runs on the first multi-GPU lease)")
def test_rccl_two_gpus_bucket_average_equals_mean_of_shard_grads(tmp_path):
    mp.spawn(_two, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in [json.load(open(tmp_path / ("t%d.json" % k))) for k in range(2)]:
        assert r["backend"] == "nccl"
        assert r["local_diff"] > 1e-3 * r["scale"]
        assert r["max_err"] <= 1e-6 * r["scale"] + 1e-9, r


@pytest.mark.skipif(_ngpu() < 2, reason="needs two GPUs (runs on the first multi-GPU lease)")
def test_async_ps_rccl_data_plane_through_epoch_boundary(tmp_path):
    """--is_sync=0 on two GPUs with the nccl backend: the server thread's RCCL
    point-to-point data plane runs while the main threads evaluate at the epoch
    boundaries (their collectives on the host group): the job completes, both
    workers' pushes land, and the final evaluation is written."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("UNET_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "train.py"),
           "--synthetic", "--is_sync", "0", "--epochs", "2", "--img_size", "64", "--in_channels", "4",
           "--batch_size", "8", "--synthetic_train", "32", "--synthetic_test", "16", "--no_checkpoint",
           "--dist_timeout_s", "120", "--checkpoint_dir", str(tmp_path / "ck"),
           "--log_jsonl", str(tmp_path / "m.jsonl")]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "Worker #1 reports job finished." in r.stdout
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len([x for x in recs if x["kind"] == "test"]) >= 1
    final = [x for x in recs if x["kind"] == "test_final"]
    assert len(final) == 1 and final[0]["step"] == 8      # 2 epochs x 4 global batches, one push each
