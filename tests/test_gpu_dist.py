"""Multi-rank data parallelism on the NATIVE backend, rehearsed on one card.

Two ranks share cuda:0 and talk over gloo (RCCL refuses two ranks on one device;
the 8-GPU node runs the same code with the nccl backend).  Each rank runs the HIP
executor's forward + backward on its own shard; the bucketed allreduce issued
between backward segments (parallel/grad_sync.py, overlapped on the side stream)
must leave every rank with the MEAN of the per-rank shard gradients -- the
reference's SyncReplicasOptimizer semantics (`test_dist.py:249-262`, SURVEY.md
§2.5).  A second check runs the same step through the non-overlapped path.
"""

import json
import os
import socket
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


def _rank(rank, world, port, out, overlap, hip_graph):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", UNET_DIST_BACKEND="gloo")
    sys.path.insert(0, ROOT)
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
    cfg = Config(batch_size=4 * world, img_size=64, in_channels=4, hip_graph=hip_graph)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=7 + rank))       # different inits ...
    D.broadcast_(flat.master, 0)                                       # ... made identical
    bounds = plan_buckets(flat, 0.25)                                  # several buckets
    be = NativeBackend(spec, flat, cfg, dev, 4, bounds)
    be.engine.repack()
    x, y = synthetic_brats(4, 64, 4, seed=100 + rank)                  # this rank's shard
    x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    # local (un-synchronised) gradient of the shard
    be.fwd_bwd(x, y, seed=5 + rank)
    torch.cuda.synchronize()
    local = flat.grad.detach().cpu().clone()
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    mean = torch.stack(gathered).mean(0)
    # the same step with the bucketed allreduce between backward segments
    sync = GradSync(flat, bounds, ctx, overlap=overlap)
    be.fwd_bwd(x, y, seed=5 + rank, on_segment=sync.on_segment)
    sync.finish()
    torch.cuda.synchronize()
    g = flat.grad.detach().cpu()
    rec = dict(rank=rank, buckets=len(bounds), max_err=(g - mean).abs().max().item(),
               scale=mean.abs().max().item(), local_diff=(local - mean).abs().max().item())
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(rec, f)
    D.destroy()


@pytest.mark.parametrize("overlap,hip_graph", [(True, True), (False, False)])
def test_native_two_ranks_bucket_average_equals_mean_of_shard_grads(tmp_path, overlap, hip_graph):
    world = 2
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path), overlap, hip_graph), nprocs=world, join=True)
    recs = [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(world)]
    for r in recs:
        assert r["buckets"] >= 3
        # the shards differ, so the local gradients differ from the mean ...
        assert r["local_diff"] > 1e-3 * r["scale"]
        # ... and after the bucketed allreduce every rank holds exactly the mean
        assert r["max_err"] <= 1e-6 * r["scale"] + 1e-9, r


def _ps_rank(rank, world, port, out, steps, batch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", UNET_DIST_BACKEND="gloo")
    sys.path.insert(0, ROOT)
    import time
    import statistics
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.async_ps import AsyncPS, DeviceParameterServer
    from unet_distributed_amd.runtime.backends import NativeBackend
    from unet_distributed_amd.runtime.params import FlatParams
    ctx = D.init("cuda", "auto", 120)
    dev = ctx.device
    cfg = Config(batch_size=batch * world, img_size=128, in_channels=4, is_sync=0)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=7))
    be = NativeBackend(spec, flat, cfg, dev, batch)
    be.engine.repack()
    ps = AsyncPS(flat, cfg, ctx, repack=be.engine.repack)
    x, y = synthetic_brats(batch, 128, 4, seed=100 + rank)
    x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    t_comp, t_ps = [], []
    for i in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        be.fwd_bwd(x, y, seed=i * world + rank)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ps.push_pull()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_comp.append(t1 - t0)
        t_ps.append(t2 - t1)
    ps.finish()
    D.barrier()
    D.broadcast_(flat.master, 0)
    torch.cuda.synchronize()
    rec = dict(rank=rank, comp_ms=1e3 * statistics.median(t_comp[2:]), ps_ms=1e3 * statistics.median(t_ps[2:]),
               device_server=isinstance(ps.server, DeviceParameterServer) if rank == 0 else None,
               step=flat.global_step, finite=bool(torch.isfinite(flat.master).all().item()))
    with open(os.path.join(out, "ps%d.json" % rank), "w") as f:
        json.dump(rec, f)
    D.destroy()


def test_async_ps_device_server_two_ranks_one_card(tmp_path):
    """--is_sync=0 with the GPU-resident parameter server: rank 0's server thread runs
    TF-Adam as one native launch per push on its own stream; 2 ranks x 8 steps all
    land (PS global_step 16); the push/pull round trip (gloo data plane staged through
    host buffers on one card) is recorded against the compute step."""
    world, steps = 2, 8
    mp.spawn(_ps_rank, args=(world, _free_port(), str(tmp_path), steps, 256), nprocs=world, join=True)
    recs = [json.load(open(tmp_path / ("ps%d.json" % r))) for r in range(world)]
    assert recs[0]["device_server"] is True
    assert all(r["finite"] for r in recs)
    assert recs[0]["step"] == world * steps
    print("async PS: compute %.2f ms, push/pull %.2f ms (rank 0, in-process) / %.2f ms (rank 1, gloo)"
          % (recs[0]["comp_ms"], recs[0]["ps_ms"], recs[1]["ps_ms"]))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "async_ps_timing.json"), "w") as f:
            json.dump(recs, f)


def test_bench_py_two_ranks_one_card_native():
    """The exact multi-GPU bench command the driver's 8-GPU lease runs
    (`torch.distributed.run --nproc-per-node N bench.py --gpus N`), at N = 2 with both
    ranks on cuda:0 over gloo (UNET_DIST_BACKEND=gloo; RCCL refuses two ranks on one
    device): the native executor, HIP graphs, the side-stream bucket allreduces, the
    MAX-over-ranks timing and the N > 1 comm diagnostics all execute before any 8-GPU
    run does."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_distributed_cpu import _run_bench, bench_record, check_multirank_bench
    r = _run_bench(["--per_gpu_batch", "64", "--steps", "3", "--warmup", "2"], timeout=300,
                   env_extra=dict(UNET_DIST_BACKEND="gloo"))
    assert r.returncode == 0, r.stdout[-3000:]
    rec = bench_record(r.stdout)
    check_multirank_bench(rec, 2)
    assert rec["config"]["backend"] == "native" and rec["comm"]["backend"] == "gloo"
    assert rec["dtype"] == "bf16" and rec["config"]["img_size"] == 128 and rec["config"]["in_channels"] == 4
    print("2-rank one-card bench:", json.dumps(rec["comm"]))
