"""Process-group lifecycle (one process per GPU, torch.distributed over RCCL).

Replaces the reference's TF gRPC cluster (`test_dist.py:14-25` host tables,
`test_dist.py:93-103` role-by-IP, `test_dist.py:130-131` ClusterSpec/Server):

* rendezvous is env:// (``MASTER_ADDR``/``MASTER_PORT``/``RANK``/``WORLD_SIZE``
  as set by ``torch.distributed.run`` or our ``launch.py``); the reference's
  chief is rank 0;
* backend ``nccl`` (= RCCL on ROCm, over xGMI inside an MI355X node) for GPU
  tensors, ``gloo`` for the CPU plumbing configuration;
* a finite collective timeout plus async error handling make a dead rank fail
  the job fast instead of blocking forever like the reference's done-queue
  (`test_dist.py:158-160`).
"""

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


class DistContext:
    def __init__(self):
        self.rank = 0
        self.world_size = 1
        self.local_rank = 0
        self.backend = None
        self.initialized = False
        self.device = torch.device("cpu")

    @property
    def is_chief(self) -> bool:
        return self.rank == 0


_CTX = DistContext()


def context() -> DistContext:
    return _CTX


def init(device_pref: str = "auto", backend: str = "auto", timeout_s: float = 300.0,
         force: bool = False) -> DistContext:
    """``force``: create the process group even at WORLD_SIZE 1 (RCCL accepts a
    one-rank communicator), so every nccl-only code path -- ``device_id`` binding,
    ``barrier(device_ids)``, ``ReduceOp.AVG`` buckets -- can run on a 1-GPU box."""
    ctx = _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_cuda = (device_pref == "cuda") or (device_pref == "auto" and torch.cuda.is_available())
    if use_cuda:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % max(ndev, 1))
        ctx.device = torch.device("cuda", local % max(ndev, 1))
    else:
        ctx.device = torch.device("cpu")
    ctx.rank, ctx.world_size, ctx.local_rank = rank, world, local
    if (world > 1 or force) and not dist.is_initialized():
        # UNET_DIST_BACKEND=gloo forces gloo for GPU tensors too: lets several
        # ranks share ONE card (RCCL refuses duplicate devices) to rehearse the
        # multi-rank GPU path on a 1-GPU box.
        backend = os.environ.get("UNET_DIST_BACKEND", backend)
        if backend == "auto":
            backend = "nccl" if use_cuda else "gloo"
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = ctx.device
        dist.init_process_group(**kw)
        ctx.backend = backend
        ctx.initialized = True
    elif dist.is_initialized():
        ctx.backend = dist.get_backend()
        ctx.initialized = True
    return ctx


# Host collectives (set_host_collectives): while set, the module's collectives run
# on CPU copies over this (gloo) group instead of the default one.
_HOST_GROUP = None


def set_host_collectives(group) -> None:
    """Route allreduce_* / broadcast_ / allreduce_max_scalar through ``group`` on
    CPU tensors (None restores the default group).  The async parameter server sets
    it for the run: its RCCL data plane is driven by the server thread, and the
    trainer's collectives (per-epoch evaluation, BatchNorm statistics) from the main
    thread must not be a second RCCL communicator issued concurrently with no
    cross-rank order -- a known deadlock pattern."""
    global _HOST_GROUP
    _HOST_GROUP = group


def _host(t: torch.Tensor, fn):
    h = t.detach().to("cpu", copy=True)
    fn(h, _HOST_GROUP)
    t.copy_(h)
    return t


def barrier():
    if _CTX.initialized:
        if _CTX.backend == "nccl":
            dist.barrier(device_ids=[_CTX.device.index])
        else:
            dist.barrier()


def broadcast_(t: torch.Tensor, src: int = 0):
    """In-place broadcast (rank 0 -> all); used for initial parameters and
    restored checkpoints (replaces `prepare_or_wait_for_session`, test_dist.py:361)."""
    if _CTX.initialized and _CTX.world_size > 1:
        if _HOST_GROUP is not None:
            return _host(t, lambda h, g: dist.broadcast(h, src, group=g))
        dist.broadcast(t, src)


def allreduce_sum_(t: torch.Tensor):
    if _CTX.initialized and _CTX.world_size > 1:
        if _HOST_GROUP is not None:
            return _host(t, lambda h, g: dist.all_reduce(h, op=dist.ReduceOp.SUM, group=g))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_avg_(t: torch.Tensor):
    if _CTX.initialized and _CTX.world_size > 1:
        if _HOST_GROUP is not None:
            _host(t, lambda h, g: dist.all_reduce(h, op=dist.ReduceOp.SUM, group=g))
            return t.div_(_CTX.world_size)
        if _CTX.backend == "nccl":
            dist.all_reduce(t, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            t.div_(_CTX.world_size)
    return t


def allreduce_max_scalar(x: float, device=None) -> float:
    if not (_CTX.initialized and _CTX.world_size > 1):
        return float(x)
    if _HOST_GROUP is not None:
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_HOST_GROUP)
        return float(t.item())
    t = torch.tensor([float(x)], dtype=torch.float64, device=device or _CTX.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy(orderly: bool = True):
    """Teardown.  ``orderly``: barrier first (replaces the done-queue shutdown,
    test_dist.py:498-502).  On an error path the barrier is skipped -- peers may
    already be gone and waiting for them would turn a crash into a hang."""
    if _CTX.initialized and dist.is_initialized():
        try:
            if orderly:
                barrier()
        finally:
            dist.destroy_process_group()
        _CTX.initialized = False
