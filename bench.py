"""Headline benchmark: images/sec of 2D UNet training on BraTS-shaped 128x128x4
synthetic slices (BASELINE.json metric), one process per GPU.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 8 --steps 20 --warmup 5

Each timed step is a complete training step of the flagship configuration:
device-side batch load, UNet forward (bf16 HIP kernels), Dice loss, backward,
bucketed RCCL allreduce (overlapped with backward), fused TF-Adam update.
Weak scaling: the per-GPU micro-batch is fixed (default 1024, sized from the batch sweep
in profiles/r2_batch_sweep.md: throughput saturates from 512 on; the reference's
per-worker shard is 256 = its 1024 global batch over 4 workers, `settings_dist.py:17`,
`test_dist.py:390`, and ``--per_gpu_batch 256`` reproduces it), so the global batch is
1024*N.  Random-init weights (he_uniform / glorot as the reference), synthetic data.

Rank 0 prints ONE JSON line; ``value`` is whole-job images/sec computed from the
MAX over ranks of the timed wall time.
"""

import argparse
import json
import os
import sys
import time

import torch


def _baseline_metric():
    """The headline metric name exactly as BASELINE.json states it."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "images/sec (whole node) 2D UNet BraTS 128x128x4 training"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--per_gpu_batch", type=int, default=None,
                   help="images per GPU; default 1024 for 2D (profiles/r2_batch_sweep.md: throughput "
                        "saturates from 512), 8 volumes for 3D (profiles/r3_bench_history.md 3D sweep: "
                        "2 / 4 / 8 -> 236 / 258 / 271 vol/s)")
    p.add_argument("--img_size", type=int, default=128)
    p.add_argument("--in_channels", type=int, default=4)
    p.add_argument("--dims", type=int, default=2)
    p.add_argument("--use_upsampling", action="store_true")
    p.add_argument("--norm", default="none", choices=["none", "batch", "group"])
    p.add_argument("--groups", type=int, default=8)
    p.add_argument("--backend", default="auto", choices=["auto", "native", "torch"])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp16"])
    p.add_argument("--bucket_mb", type=float, default=8.0)
    p.add_argument("--no_overlap", action="store_true")
    p.add_argument("--hip_graph", type=int, default=1,
                   help="replay fwd / bwd segments / Adam as captured HIP graphs (0: eager launches)")
    p.add_argument("--profile_dir", default="")
    p.add_argument("--dist_force", type=int, default=0,
                   help="1: create the process group and issue the bucket collectives even at one rank "
                        "(exercises the RCCL path on a 1-GPU box; the timed step then includes them)")
    p.add_argument("--comm_diag", type=int, default=1,
                   help="N > 1: after the timed steps, measure per-bucket allreduce time and the exposed "
                        "communication (A/B against compute-only and non-overlapped steps)")
    return p.parse_args()


class _NoComm:
    """Compute-only stand-in for GradSync (comm diagnostics A/B)."""

    def on_segment(self, i):
        pass

    def finish(self):
        pass


def comm_diagnostics(a, ctx, flat, bounds, sync_overlap, step_fn, dev):
    """Outside the timed region: per-bucket allreduce time (isolated, median of 5,
    events on the issuing stream) and the step time with overlapped / serial / no
    communication, so a multi-GPU number comes with its comm breakdown."""
    import statistics
    import torch.distributed as dist
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.grad_sync import GradSync
    out = {"backend": ctx.backend or "none", "world_size": ctx.world_size,
           "buckets_mb": [round(4.0 * (b - (bounds[i - 1] if i else 0)) / 2 ** 20, 3) for i, b in enumerate(bounds)]}
    if (ctx.world_size == 1 and not a.dist_force) or not ctx.initialized or not a.comm_diag:
        return out
    per = []
    for i in range(len(bounds)):
        t = sync_overlap._slice(i)
        samples = []
        cuda = dev.type == "cuda"
        for _ in range(5):
            D.barrier()
            if cuda:
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            t0 = time.perf_counter()
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            if cuda:
                e1.record()
                torch.cuda.synchronize()
                samples.append(e0.elapsed_time(e1))
            else:
                samples.append((time.perf_counter() - t0) * 1000.0)
        per.append(round(D.allreduce_max_scalar(statistics.median(samples), dev), 4))
    out["allreduce_ms_per_bucket"] = per
    out["allreduce_ms_total"] = round(sum(per), 4)

    def sync_dev():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def timed(sync, k=5):
        step_fn(0, sync)
        sync_dev()
        D.barrier()
        sync_dev()
        t0 = time.perf_counter()
        for i in range(k):
            step_fn(1 + i, sync)
        sync_dev()
        D.barrier()
        sync_dev()
        return D.allreduce_max_scalar((time.perf_counter() - t0) * 1000.0 / k, dev)

    t_none = timed(_NoComm())
    t_ovl = timed(sync_overlap)
    t_ser = timed(GradSync(flat, bounds, ctx, overlap=False, force=bool(a.dist_force)))
    out.update(step_ms_compute_only=round(t_none, 3), step_ms_overlapped=round(t_ovl, 3),
               step_ms_serial_comm=round(t_ser, 3), exposed_comm_ms=round(t_ovl - t_none, 3),
               serial_comm_ms=round(t_ser - t_none, 3))
    return out


def main():
    a = parse()
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel import dist as D
    from unet_distributed_amd.parallel.grad_sync import GradSync, plan_buckets
    from unet_distributed_amd.runtime.backends import make_backend
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.runtime.trainer import _NativeOpt
    from unet_distributed_amd.runtime.amp import LossScaler

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    ctx = D.init("auto", "auto", 600.0, force=bool(a.dist_force))
    N = ctx.world_size
    if world_env != a.gpus and ctx.rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (a.gpus, world_env), file=sys.stderr)
    if a.per_gpu_batch is None:
        a.per_gpu_batch = 8 if a.dims == 3 else 1024
    cfg = Config(batch_size=a.per_gpu_batch * N, in_channels=a.in_channels, img_size=a.img_size,
                 dims=a.dims, use_upsampling=a.use_upsampling, backend=a.backend, dtype=a.dtype,
                 norm=a.norm, groups=a.groups,
                 synthetic=True, no_checkpoint=True, bucket_mb=a.bucket_mb, overlap_comm=not a.no_overlap,
                 hip_graph=bool(a.hip_graph))
    dev = ctx.device
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=cfg.seed))
    D.broadcast_(flat.master, 0)
    bounds = plan_buckets(flat, cfg.bucket_mb)
    backend = make_backend(spec, flat, cfg, dev, a.per_gpu_batch, bounds)
    if hasattr(backend, "engine"):
        backend.engine.repack()
    sync = GradSync(flat, bounds, ctx, overlap=cfg.overlap_comm, force=bool(a.dist_force))
    opt = TFAdam(flat, cfg, native=_NativeOpt(backend) if hasattr(backend, "adam_step") else None)

    # two distinct synthetic batches resident on the device (per-rank shards)
    B = a.per_gpu_batch
    xs, ys = [], []
    for k in range(2):
        x, y = synthetic_brats(B, a.img_size, a.in_channels, a.dims, seed=1000 * ctx.rank + k)
        xs.append(torch.from_numpy(x).to(dev))
        ys.append(torch.from_numpy(y).to(dev))

    scaler = LossScaler(cfg.dtype, cfg.loss_scale)

    def step(i, sync=sync):
        scale = scaler.scale
        backend.fwd_bwd(xs[i % 2], ys[i % 2], seed=12345 + i, on_segment=sync.on_segment, grad_scale=scale)
        sync.finish()
        if scaler.update(flat.grad):            # fp16: finiteness check + dynamic scale (no-op in bf16)
            opt.step(grad_scale=1.0 / scale)

    for i in range(a.warmup):
        step(i)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    D.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    prof = None
    if a.profile_dir and ctx.rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    D.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.profile_dir, "trace.json"))
    dt = D.allreduce_max_scalar(dt, dev)
    imgs = a.steps * B * N
    s = backend.sums()
    i_, st, sp = [float(v) for v in s[:3].tolist()]
    dice = (2 * i_ + 1) / (st + sp + 1)
    comm = comm_diagnostics(a, ctx, flat, bounds, sync, step, dev)
    if ctx.rank == 0:
        rec = {
            "metric": (_baseline_metric()
                       if (a.dims, a.img_size, a.in_channels) == (2, 128, 4) else
                       "images/sec (whole node) %dD UNet %s x%d training"
                       % (a.dims, "x".join([str(a.img_size)] * a.dims), a.in_channels)),
            "value": round(imgs / dt, 2),
            "unit": "images/sec",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (BraTS-shaped %s x%d %s, random-init weights)"
                    % ("x".join([str(a.img_size)] * a.dims), a.in_channels, "slices" if a.dims == 2 else "volumes"),
            "config": {"model": "unet%dd-%s%s (base 32, depth 4, %d params)"
                                % (a.dims, "upsampling" if a.use_upsampling else "transposed",
                                   "" if a.norm == "none" else "-" + a.norm + "norm", spec.num_params()),
                       "global_batch": B * N, "per_gpu_batch": B, "seq_len": None,
                       "img_size": a.img_size, "in_channels": a.in_channels,
                       "parallelism": "dp%d" % N, "backend": backend.name},
            "train_dice_last_batch": round(dice, 5),
            "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2) if torch.cuda.is_available() else None,
            "comm": comm,
        }
        print(json.dumps(rec), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
