"""Asynchronous parameter-server mode (``--is_sync=0``).

Reference behaviour (`test_dist.py:264-267`): without
SyncReplicasOptimizer every worker's ``apply_gradients`` runs straight on the
PS variables -- Hogwild-style, no barrier, each worker computing on whatever
(possibly stale) weights it last pulled; ``global_step`` advances once per
worker step.  The done-queue (`test_dist.py:106-119,498-502`) tells the PS when
every worker has finished.

Emulation on a single MI355X node: rank 0 additionally hosts the parameter
server in a background thread that owns the fp32 master weights and the TF-Adam
state (CPU, like the reference's PS).  Every rank -- rank 0 included -- trains
on its shard and, after each backward, pushes its gradient to the server and
pulls the freshly updated weights.  Transport is a dedicated gloo process group
(point-to-point isend/recv from any source); rank 0's own worker talks to the
server in-process.  Message tags: GRAD (worker -> PS, followed by the gradient
tensor), DONE (worker -> PS, the done-queue token).
"""

import threading
from typing import Optional

import torch
import torch.distributed as dist

from ..runtime.optim import BETA1, BETA2, adam_reference_, learning_rate

TAG_HDR, TAG_GRAD, TAG_PARAMS = 11, 12, 13
MSG_GRAD, MSG_DONE = 1, 2


class ParameterServer:
    """TF-Adam on the master weights, applied in gradient arrival order."""

    def __init__(self, flat, cfg):
        self.w = flat.master.detach().to("cpu", torch.float32).clone()
        self.m = flat.m.detach().to("cpu", torch.float32).clone()
        self.v = flat.v.detach().to("cpu", torch.float32).clone()
        self.cfg = cfg
        self.step = flat.global_step
        self.b1p, self.b2p = flat.beta1_power, flat.beta2_power
        self.lock = threading.Lock()

    def apply(self, g: torch.Tensor, out: torch.Tensor) -> int:
        """One Hogwild update; copies the new weights into ``out``, returns global_step."""
        with self.lock:
            lr = learning_rate(self.cfg, self.step)
            adam_reference_(self.w, g, self.m, self.v, lr, self.b1p, self.b2p)
            self.b1p *= BETA1
            self.b2p *= BETA2
            self.step += 1
            out.copy_(self.w)
            return self.step


class AsyncPS:
    def __init__(self, flat, cfg, ctx, repack=None):
        self.flat = flat
        self.cfg = cfg
        self.ctx = ctx
        self.repack = repack
        self.rank, self.world = ctx.rank, ctx.world_size
        self.group = dist.new_group(backend="gloo")
        self.server: Optional[ParameterServer] = None
        self.thread = None
        self.gbuf = torch.zeros(flat.numel, dtype=torch.float32)
        self.pbuf = torch.zeros(flat.numel + 2, dtype=torch.float32)
        self.ps_step = flat.global_step
        self.local_steps = 0
        if self.rank == 0:
            self.server = ParameterServer(flat, cfg)
            self.thread = threading.Thread(target=self._serve, daemon=True)
            self.thread.start()

    # ------------------------------------------------------------- server (rank 0)
    def _serve(self):
        done = 0
        hdr = torch.zeros(2, dtype=torch.int64)
        g = torch.zeros(self.flat.numel, dtype=torch.float32)
        w = torch.zeros(self.flat.numel + 2, dtype=torch.float32)
        while done < self.world - 1:
            src = dist.recv(hdr, src=None, group=self.group, tag=TAG_HDR)
            if int(hdr[0]) == MSG_DONE:
                done += 1
                print("Worker #{} reports job finished.".format(src), flush=True)
                continue
            dist.recv(g, src=src, group=self.group, tag=TAG_GRAD)
            step = self.server.apply(g, w[:-2])
            w[-2] = float(step & 0xFFFFFF)          # step split in two exact fp32 halves
            w[-1] = float(step >> 24)
            dist.send(w, dst=src, group=self.group, tag=TAG_PARAMS)

    # ------------------------------------------------------------- worker side
    def push_pull(self):
        """Send this worker's gradient, receive the PS weights (one async step)."""
        self.gbuf.copy_(self.flat.grad, non_blocking=False)
        if self.rank == 0:
            self.ps_step = self.server.apply(self.gbuf, self.pbuf[:-2])
        else:
            hdr = torch.tensor([MSG_GRAD, self.local_steps], dtype=torch.int64)
            dist.send(hdr, dst=0, group=self.group, tag=TAG_HDR)
            dist.send(self.gbuf, dst=0, group=self.group, tag=TAG_GRAD)
            dist.recv(self.pbuf, src=0, group=self.group, tag=TAG_PARAMS)
            self.ps_step = int(self.pbuf[-2].item()) | (int(self.pbuf[-1].item()) << 24)
        self.flat.master.copy_(self.pbuf[:-2].to(self.flat.master.device))
        self.local_steps += 1
        self.flat.global_step = self.ps_step      # the PS's shared global_step, as in TF
        if self.repack is not None:
            self.repack()

    def skip_step(self):
        """A local iteration that pushed nothing (fp16 overflow): it still counts, so
        every rank's epoch boundaries -- and the collectives evaluate() issues there --
        stay in lockstep."""
        self.local_steps += 1

    def snapshot_into_flat(self):
        """Copy the PS state (weights, Adam slots, step, beta powers) into ``flat``
        on rank 0 -- used before a checkpoint save so the bundle is the PS's."""
        if self.server is None:
            return
        sv = self.server
        with sv.lock:
            dev = self.flat.master.device
            self.flat.master.copy_(sv.w.to(dev))
            self.flat.m.copy_(sv.m.to(dev))
            self.flat.v.copy_(sv.v.to(dev))
            self.flat.global_step = sv.step
            self.flat.beta1_power, self.flat.beta2_power = sv.b1p, sv.b2p

    def finish(self):
        """Done-queue shutdown: workers enqueue a token; the PS waits for all of them."""
        if self.rank != 0:
            hdr = torch.tensor([MSG_DONE, 0], dtype=torch.int64)
            dist.send(hdr, dst=0, group=self.group, tag=TAG_HDR)
        elif self.thread is not None:
            self.thread.join()
            self.snapshot_into_flat()
            if self.repack is not None:
                self.repack()
