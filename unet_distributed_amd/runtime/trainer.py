"""Training runtime: the reference's worker ``main()`` re-designed for MI355X.

Reference flow (`test_dist.py:121-508`): build the graph,
SyncReplicasOptimizer over a parameter server, Supervisor-managed session with
auto-restore, a hot loop that shards each global batch over the workers, chief
duties (summaries, per-epoch evaluation, ``last_good_model`` save, TensorBoard,
SavedModel export), and a done-queue shutdown.

Here: one process per GPU; full replicas; bucketed RCCL allreduce overlapped
with the native backward; fused TF-Adam on every rank; rank 0 does logging,
evaluation reporting, checkpoints and export; checkpoints auto-resume; a dead
rank fails the job through collective timeouts.  Fixes of reference quirks are
listed in SURVEY.md Appendix Q and noted inline.
"""

import json
import math
import os
import sys
import time
from typing import Optional

import numpy as np
import torch

from .. import settings
from ..data import datasets
from ..data.loader import DeviceFeeder
from ..models import reference
from ..models.spec import spec_from_config
from ..ops import losses
from ..parallel import dist as D
from ..parallel.async_ps import AsyncPS
from ..parallel.grad_sync import GradSync, plan_buckets
from ..utils import checkpoint as ckpt
from ..utils.metrics import MetricLogger
from .amp import LossScaler
from .backends import make_backend
from .optim import TFAdam, learning_rate
from .params import FlatParams


class FaultInjected(RuntimeError):
    pass


class _Ranges:
    """roctx ranges (torch.cuda.nvtx is backed by roctx on ROCm builds) plus
    torch.profiler record_function labels, so rocprofv3 --marker-trace and the
    Chrome trace both show forward_backward / grad_sync / optimizer."""

    def __init__(self, on: bool):
        self.on = on

    class _R:
        def __init__(self, name, on):
            self.name, self.on, self.rf = name, on, None

        def __enter__(self):
            if self.on:
                try:
                    torch.cuda.nvtx.range_push(self.name)
                except Exception:
                    pass
                self.rf = torch.autograd.profiler.record_function(self.name)
                self.rf.__enter__()

        def __exit__(self, *a):
            if self.on:
                self.rf.__exit__(*a)
                try:
                    torch.cuda.nvtx.range_pop()
                except Exception:
                    pass

    def __call__(self, name):
        return self._R(name, self.on)


def _make_profiler(cfg, rank, logdir):
    """--profile: torch.profiler (roctracer-backed HIP kernel trace) over local
    steps [a, b) of --profile_steps a,b; Chrome trace per rank in logdir/profile."""
    a, b = [int(v) for v in cfg.profile_steps.split(",")]
    out = os.path.join(logdir, "profile")
    os.makedirs(out, exist_ok=True)

    def ready(prof):
        path = os.path.join(out, "trace_rank%d.json" % rank)
        prof.export_chrome_trace(path)
        if rank == 0:
            print("profiler: wrote %s" % path, flush=True)
            print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=25), flush=True)

    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    return torch.profiler.profile(activities=acts,
                                  schedule=torch.profiler.schedule(wait=max(a - 1, 0), warmup=1 if a > 0 else 0,
                                                                   active=max(b - a, 1), repeat=1),
                                  on_trace_ready=ready)


def metrics_from_sums(s: torch.Tensor, npix: int, cfg) -> dict:
    i, st, sp, bce = [float(v) for v in s.tolist()]
    m = losses.metrics_from_sums(i, st, sp)
    if cfg.loss == "dice_bce":
        m["loss"] += cfg.bce_weight * bce / max(npix, 1)
    return m


class Trainer:
    def __init__(self, cfg):
        self.cfg = cfg
        self.ctx = D.init(cfg.device, cfg.dist_backend, cfg.dist_timeout_s)
        self.device = self.ctx.device
        self.rank, self.world = self.ctx.rank, self.ctx.world_size
        self.is_chief = self.ctx.is_chief
        if cfg.batch_size % self.world:
            raise SystemExit("--batch_size %d must be divisible by the world size %d"
                             % (cfg.batch_size, self.world))
        self.per_rank = cfg.batch_size // self.world
        torch.manual_seed(cfg.seed)
        self.spec = spec_from_config(cfg)
        self.flat = FlatParams(self.spec, device=self.device)
        self.flat.load_dict(reference.init_params(self.spec, seed=cfg.seed))
        self.bounds = plan_buckets(self.flat, cfg.bucket_mb)
        self.backend = make_backend(self.spec, self.flat, cfg, self.device, self.per_rank, self.bounds)
        extra = getattr(self.backend, "state", {}) or {}
        self.ckpt = ckpt.CheckpointManager(cfg, self.flat, self.is_chief, extra_state=extra)
        self.restored = False
        if cfg.resume and self.is_chief and not cfg.no_checkpoint:
            self.restored = self.ckpt.restore_latest()
        self._broadcast_state()
        # --is_sync=0: Hogwild updates through a parameter server (test_dist.py:264-267)
        self.async_ps = None
        if cfg.is_sync == 0 and self.world > 1:
            engine = getattr(self.backend, "engine", None)
            self.async_ps = AsyncPS(self.flat, cfg, self.ctx,
                                    repack=engine.repack if engine is not None else None)
        if self.async_ps is not None and self.is_chief:
            self.ckpt.pre_save = self.async_ps.snapshot_into_flat
        self.sync = GradSync(self.flat, self.bounds, self.ctx, overlap=cfg.overlap_comm)
        native_opt = self.backend if hasattr(self.backend, "adam_step") else None
        self.opt = TFAdam(self.flat, cfg, native=_NativeOpt(native_opt) if native_opt else None)
        self.scaler = LossScaler(cfg.dtype, cfg.loss_scale)
        self.log = MetricLogger(cfg, self.is_chief, self.ckpt.logdir)
        self.ranges = _Ranges(cfg.profile)
        self.tb_proc = None
        if cfg.launch_tensorboard and self.is_chief:
            import shutil
            import subprocess
            exe = shutil.which("tensorboard")
            if exe:     # test_dist.py:375-378
                self.tb_proc = subprocess.Popen([exe, "--logdir", self.ckpt.logdir])
            else:
                print("tensorboard is not installed; event files are in %s" % self.ckpt.logdir)
        self._load_data()

    # ------------------------------------------------------------------ setup
    def _broadcast_state(self):
        f = self.flat
        for t in (f.master, f.m, f.v):
            D.broadcast_(t, 0)
        meta = torch.tensor([f.global_step, f.beta1_power, f.beta2_power, int(self.restored)],
                            dtype=torch.float64, device=self.device)
        D.broadcast_(meta, 0)
        f.global_step = int(meta[0].item())
        f.beta1_power = float(meta[1].item())
        f.beta2_power = float(meta[2].item())
        self.restored = bool(meta[3].item())
        self._broadcast_extra()
        if hasattr(self.backend, "engine"):
            self.backend.engine.repack()

    def _extra_state(self):
        return getattr(self.backend, "state", None) or {}

    def _broadcast_extra(self):
        """Non-trainable state (BatchNorm moving statistics) from rank 0: after a
        resume only rank 0 restored it, and every rank must evaluate with it."""
        for k in sorted(self._extra_state()):
            D.broadcast_(self._extra_state()[k], 0)

    def _average_extra(self):
        """Replica-average the BatchNorm moving statistics (each rank tracks them over
        its own shard; the reference's PS-hosted variables are shared by all workers)."""
        st = self._extra_state()
        if self.world == 1 or not st:
            return
        for k in sorted(st):
            D.allreduce_sum_(st[k])
            st[k].mul_(1.0 / self.world)

    def _load_data(self):
        cfg = self.cfg
        if cfg.synthetic:
            n_tr = max(cfg.synthetic_train, cfg.batch_size)
            self.x_train, self.y_train = datasets.synthetic_brats(n_tr, cfg.img_size, cfg.in_channels,
                                                                  cfg.dims, seed=cfg.seed,
                                                                  difficulty=cfg.synthetic_difficulty)
            self.x_test, self.y_test = datasets.synthetic_brats(cfg.synthetic_test, cfg.img_size,
                                                                cfg.in_channels, cfg.dims, seed=cfg.seed + 1,
                                                                difficulty=cfg.synthetic_difficulty)
        else:
            xi, yi = datasets.load_data(cfg.data_path, "_train")
            self.x_train, self.y_train = datasets.update_channels(xi, yi, cfg.in_channels, cfg.out_channels, cfg.mode)
            xi, yi = datasets.load_data(cfg.data_path, "_test")
            self.x_test, self.y_test = datasets.update_channels(xi, yi, cfg.in_channels, cfg.out_channels, cfg.mode)
        if self.is_chief:
            print("Training images shape: {}".format(self.x_train.shape))
            print("Training masks shape:  {}".format(self.y_train.shape))
            print("Testing images shape:  {}".format(self.x_test.shape))
            print("Testing masks shape:   {}".format(self.y_test.shape))
        self.sampler = datasets.EpochSampler(len(self.x_train), cfg.batch_size, self.rank, self.world, cfg.seed)
        self.num_batches = self.sampler.num_batches
        self.feeder = DeviceFeeder(self.x_train, self.y_train, self.per_rank, self.device,
                                   threads=min(cfg.num_threads, 16), mode=cfg.data_on_device)
        if self.is_chief:
            print("Training data: %s" % ("resident in device memory" if self.feeder.resident
                                         else "streamed from host (pinned, double-buffered)"))

    def _batch(self, idx: np.ndarray):
        # native backend + resident data: the backend gathers the batch itself (one
        # gather+cast kernel into its input buffers, no fp32 batch copy)
        return self.feeder.get(idx, lazy=self.backend.name == "native")

    # ------------------------------------------------------------------ eval
    def evaluate(self) -> dict:
        """Per-epoch test metrics: every full per-rank batch, sharded over ranks,
        batch metrics averaged over ALL batches (fixes the under-count of Q7)."""
        n = len(self.x_test)
        B = self.per_rank
        nbatches = n // B
        acc = torch.zeros(5, dtype=torch.float64, device=self.device)
        for b in range(self.rank, nbatches, self.world):
            x = torch.from_numpy(np.ascontiguousarray(self.x_test[b * B:(b + 1) * B])).to(self.device)
            y = torch.from_numpy(np.ascontiguousarray(self.y_test[b * B:(b + 1) * B])).to(self.device)
            m = metrics_from_sums(self.backend.eval_sums(x, y), y.numel(), self.cfg)
            acc += torch.tensor([m["loss"], m["dice"], m["sensitivity"], m["specificity"], 1.0],
                                dtype=torch.float64, device=self.device)
        D.allreduce_sum_(acc)
        cnt = max(acc[4].item(), 1.0)
        return {"loss": acc[0].item() / cnt, "dice": acc[1].item() / cnt,
                "sensitivity": acc[2].item() / cnt, "specificity": acc[3].item() / cnt,
                "batches": int(acc[4].item())}

    # ------------------------------------------------------------------ step
    def _poison_due(self, step: int) -> bool:
        """--fault_inject_overflow_step: this rank's gradient is made non-finite (fp16
        overflow drill) ONCE, at the first iteration of the given step.  (A skipped
        step does not advance global_step, so the retried iteration carries the same
        step number: a step-number test alone would poison every retry forever.)"""
        c = self.cfg
        return (not getattr(self, "_poisoned", False) and c.fault_inject_overflow_step == step
                and c.fault_inject_rank in (-1, self.rank))

    def _poison(self) -> None:
        self._poisoned = True
        self.flat.grad[0] = float("inf")

    def train_step(self, x, y, seed: int, step: int = -2) -> None:
        R = self.ranges
        scale = self.scaler.scale
        poison = self._poison_due(step)
        if self.async_ps is not None:
            with R("forward_backward"):
                self.backend.fwd_bwd(x, y, seed, on_segment=None, grad_scale=scale)
            if poison:
                self._poison()
            if self.scaler.enabled:
                if not self.scaler.update(self.flat.grad):
                    self.async_ps.skip_step()   # fp16 overflow: nothing is pushed, the
                    return                      # iteration still counts (lockstep evals)
                self.flat.grad.mul_(1.0 / scale)
            with R("ps_push_pull"):
                self.async_ps.push_pull()
            return
        on_segment = self.sync.on_segment
        if poison:
            # sync mode: poison inside the bucket hook, on the hook's stream, BEFORE the
            # allreduce of the bucket that holds flat offset 0 is issued -- so every rank
            # sees the same non-finite average and skips the step together (a write
            # after fwd_bwd would race the in-flight allreduce)
            def on_segment(i, _f=self.sync.on_segment):
                if i == 0:
                    self._poison()
                _f(i)
        with R("forward_backward"):
            self.backend.fwd_bwd(x, y, seed, on_segment=on_segment, grad_scale=scale)
        if poison and not getattr(self, "_poisoned", False):
            self._poison()                      # backend without bucket hooks
        with R("grad_sync"):
            self.sync.finish()
        if not self.scaler.update(self.flat.grad):
            return                              # fp16 overflow: step skipped, scale halved
        with R("optimizer"):
            self.opt.step(grad_scale=1.0 / scale)

    def check_sync(self):
        """Cross-rank parameter checksum (detects DP divergence)."""
        if self.world == 1:
            return
        s = self.flat.master.double().sum().reshape(1)
        mx, mn = s.clone(), s.clone()
        import torch.distributed as dist
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        if (mx - mn).abs().item() > 1e-6 * max(1.0, abs(mx.item())):
            raise RuntimeError("replica divergence detected at step %d: %g vs %g"
                               % (self.flat.global_step, mn.item(), mx.item()))

    def run(self) -> dict:
        cfg = self.cfg
        total = cfg.steps if cfg.steps > 0 else self.num_batches * cfg.epochs
        step = self.flat.global_step
        if self.async_ps is not None:
            # async: the PS global_step advances once per WORKER step, so each rank
            # runs its share of the remaining steps; the loop below then counts
            # local iterations (identical on every rank -> collectives line up).
            total = -(-(total - step) // self.world)
            step = 0
        if self.is_chief:
            print("I am chief worker with task #0 (world size %d, backend %s, device %s)"
                  % (self.world, self.backend.name, self.device))
            if self.restored:
                print("Restored checkpoint at global_step %d" % step)
        epoch = step // self.num_batches
        epoch_idx = self.sampler.epoch_indices(epoch)
        t_last = time.time()
        imgs_since = 0
        last_metrics = {}
        prof = _make_profiler(cfg, self.rank, self.ckpt.logdir) if cfg.profile else None
        if prof is not None:
            prof.start()
        while step < total:
            batch_idx = step % self.num_batches
            if batch_idx == 0 and step // self.num_batches != epoch:
                epoch = step // self.num_batches
                epoch_idx = self.sampler.epoch_indices(epoch)     # reshuffle (test_dist.py:449-452)
            x, y = self._batch(epoch_idx[batch_idx])
            if cfg.fault_inject_step >= 0 and step == cfg.fault_inject_step and \
                    (cfg.fault_inject_rank < 0 or cfg.fault_inject_rank == self.rank):
                raise FaultInjected("fault injected at step %d on rank %d" % (step, self.rank))
            # dropout stream per (step, rank): every replica draws its own masks, as the
            # reference's independent TF workers do (the hash depends only on the element
            # index, the seed and the layer)
            self.train_step(x, y, seed=cfg.seed * 1000003 + step * self.world + self.rank, step=step)
            if prof is not None:
                prof.step()
            step = self.async_ps.local_steps if self.async_ps is not None else self.flat.global_step
            imgs_since += cfg.batch_size
            if cfg.check_sync_every and step % cfg.check_sync_every == 0 and self.async_ps is None:
                self.check_sync()
            if step % cfg.log_every == 0 or step == total:
                if self.device.type == "cuda":
                    torch.cuda.synchronize()
                dt = time.time() - t_last
                m = metrics_from_sums(self.backend.sums(), x.npix if y is None else y.numel(), cfg)
                m["images_per_sec"] = imgs_since / max(dt, 1e-9)
                m["lr"] = learning_rate(cfg, step)
                m["percent_complete"] = 100.0 * step / total
                imgs = None
                if self.is_chief and self.log.events is not None and hasattr(self.backend, "summary_images"):
                    imgs = self.backend.summary_images(self.log.max_images)
                self.log.train(self.flat.global_step, m, total, images=imgs)
                last_metrics = m
                t_last, imgs_since = time.time(), 0
            if step % self.num_batches == 0:
                # end of an epoch: evaluate, report, keep last_good_model (test_dist.py:407-446)
                self._average_extra()
                tm = self.evaluate()
                self.log.test(step, tm, step // self.num_batches, cfg.epochs)
                if self.is_chief:
                    self.ckpt.save_last_good()
            self.ckpt.maybe_save()
        if prof is not None:
            prof.stop()
        if self.async_ps is not None:
            self.async_ps.finish()              # done-queue: PS waits for every worker
            D.barrier()
            D.broadcast_(self.flat.master, 0)   # final PS weights to every replica
            if hasattr(self.backend, "engine"):
                self.backend.engine.repack()
            step = self.flat.global_step
        self._average_extra()
        final = self.evaluate()
        self.log.test(step, final, step // max(self.num_batches, 1), cfg.epochs, final=True)
        if self.is_chief:
            self.ckpt.save(); self.ckpt.save_last_good()
            if cfg.export:
                d = ckpt.export_model(cfg, self.spec, self.flat,
                                         extra_state=getattr(self.backend, "state", None))
                print("Saved final model to directory: {}".format(d))
        self.log.close()
        if self.tb_proc is not None:
            self.tb_proc.terminate()            # test_dist.py:496
        return {"train": last_metrics, "test": final, "global_step": step}


class _NativeOpt:
    def __init__(self, backend):
        self.backend = backend

    def adam_step(self, lr, b1p, b2p, grad_scale):
        self.backend.adam_step(lr, b1p, b2p, grad_scale)


def main(argv=None) -> int:
    from ..config import parse_args
    cfg = parse_args(argv)
    if cfg.serialize_kernels:       # must precede the first HIP call
        os.environ["AMD_SERIALIZE_KERNEL"] = "3"
        os.environ["HIP_LAUNCH_BLOCKING"] = "1"
    if cfg.deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)
    for k in ("http_proxy", "https_proxy"):
        os.environ.pop(k, None)                 # Q5: the reference del's these unconditionally
    tr = Trainer(cfg)
    try:
        tr.run()
    except BaseException:
        D.destroy(orderly=False)
        raise
    D.destroy()
    if tr.is_chief:
        print("\n\nFinished work on this node.")
    return 0
