"""Bucketed gradient allreduce overlapped with backward.

The reference aggregates worker gradients in SyncReplicasOptimizer's
parameter-server accumulators (`test_dist.py:249-262`): every worker pushes
31 MB of gradients to the PS and pulls 31 MB of weights per step (SURVEY.md
§2.6 X1/X2).  Here every rank keeps a full replica and the gradients are
averaged with RCCL ``allreduce(AVG)`` — mathematically the same update
("mean of N worker gradients, then one Adam step").

Buckets are contiguous slices of the flat gradient buffer (which is laid out
in backward-ready order), cut at layer boundaries.  The native executor ends
a backward plan segment exactly where a bucket's last layer finished, and we
launch that bucket's allreduce immediately (``async_op=True``): RCCL runs on
its own HIP stream, ordered after the segment's kernels, while the compute
stream continues with the next layers.  ``finish()`` makes the compute stream
wait for all buckets before the optimizer.

Bucket sizing for MI355X xGMI: 8 GPUs are fully connected by 7 links of
~153 GB/s each.  RCCL spreads a ring allreduce over several channels/links,
so per-message latency (~10-30 us) rather than bandwidth dominates for these
sizes; a handful of 4-16 MB buckets keeps launches few while still leaving
only a small exposed tail (the encoder's last ~4.5 MB).
Status: this sizing is reasoned, not tuned -- no multi-rank RCCL run on xGMI hardware exists yet
(one-rank runs time the per-bucket collectives: 0.014-0.017 ms each, `bench.py --dist_force 1`,
profiles/r6_configs.md); `--bucket_mb` is the knob once an 8-GPU node measures it.
"""

from typing import List

import torch
import torch.distributed as dist

from ..models.spec import UNetSpec
from .dist import DistContext


def plan_buckets(flat, bucket_mb: float, tail_mb: float = 4.0) -> List[int]:
    """Return flat-buffer element offsets that END each bucket (layer aligned)."""
    target = max(1, int(bucket_mb * (1 << 20) / 4))
    # group variables by layer (contiguous in the flat buffer)
    layers = []
    for name, shape, off, n in flat.entries:
        lname = name.split("/")[0]
        if layers and layers[-1][0] == lname:
            layers[-1][2] = off + n
        else:
            layers.append([lname, off, off + n])
    bounds = []
    start = 0
    for i, (lname, s, e) in enumerate(layers):
        end_pad = layers[i + 1][1] if i + 1 < len(layers) else flat.numel
        if end_pad - start >= target:
            bounds.append(end_pad)
            start = end_pad
    if not bounds or bounds[-1] != flat.numel:
        bounds.append(flat.numel)
    # keep the exposed tail bucket small: split the last bucket if it is large
    if len(bounds) >= 1:
        last_start = bounds[-2] if len(bounds) >= 2 else 0
        tail_target = int(tail_mb * (1 << 20) / 4)
        if flat.numel - last_start > 2 * tail_target:
            cut = None
            for lname, s, e in layers:
                if s > last_start and flat.numel - s <= tail_target:
                    cut = s
                    break
            if cut is not None and cut > last_start:
                bounds.insert(len(bounds) - 1, cut)
    return bounds


class GradSync:
    def __init__(self, flat, bounds: List[int], ctx: DistContext, overlap: bool = True, force: bool = False):
        """``force``: issue the bucket collectives even on a one-rank process group
        (``dist.init(force=True)``), so the RCCL bucket path runs on a 1-GPU box."""
        self.flat = flat
        self.bounds = list(bounds)
        self.ctx = ctx
        self.overlap = overlap
        self.works = []
        self.issued = set()
        self.world = ctx.world_size if ctx.initialized else 1
        self.active = ctx.initialized and (self.world > 1 or force)
        self.avg_native = ctx.backend == "nccl"

    def _slice(self, i):
        s = 0 if i == 0 else self.bounds[i - 1]
        return self.flat.grad[s:self.bounds[i]]

    def on_segment(self, i: int):
        """Called right after backward segment i (covering bucket i) was enqueued, on
        the stream the segment's gradients are ordered on (the executor's side stream
        once it has joined the dgrad chain): the collective is ordered after them, and
        finish() orders the caller's stream after the collective (work.wait())."""
        if not self.active:
            return
        self.issued.add(i)
        t = self._slice(i)
        op = dist.ReduceOp.AVG if self.avg_native else dist.ReduceOp.SUM
        if self.overlap:
            self.works.append((i, dist.all_reduce(t, op=op, async_op=True)))
        else:
            dist.all_reduce(t, op=op)
            if not self.avg_native:
                t.div_(self.world)

    def sync_all(self):
        """Non-overlapped path: allreduce every bucket now."""
        for i in range(len(self.bounds)):
            self.on_segment(i)
        self.finish()

    def finish(self):
        # a bucket the backend did not hand over (fewer backward segments than buckets)
        # is reduced now: every replica must end the step with the same gradient
        for i in range(len(self.bounds)):
            if self.active and i not in self.issued:
                self.on_segment(i)
        self.issued = set()
        for i, w in self.works:
            w.wait()
            if not self.avg_native:
                self._slice(i).div_(self.world)
        self.works = []
