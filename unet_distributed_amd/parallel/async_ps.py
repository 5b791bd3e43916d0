"""Asynchronous parameter-server mode (``--is_sync=0``).

Reference behaviour (`test_dist.py:264-267`): without
SyncReplicasOptimizer every worker's ``apply_gradients`` runs straight on the
PS variables -- Hogwild-style, no barrier, each worker computing on whatever
(possibly stale) weights it last pulled; ``global_step`` advances once per
worker step.  The done-queue (`test_dist.py:106-119,498-502`) tells the PS when
every worker has finished.

Emulation on an MI355X node: rank 0 additionally hosts the parameter server in a
background thread.  On a GPU the server state (fp32 weights + TF-Adam slots) is
resident in rank 0's HBM and every update is ONE launch of the native fused Adam
kernel on a dedicated server stream (``DeviceParameterServer``); without a GPU it
is the CPU reference (``ParameterServer``).  Every rank -- rank 0 included --
trains on its shard and, after each backward, pushes its gradient and pulls the
freshly updated weights:

* control plane: a gloo group carries 16-byte headers (any-source receive, so the
  server serves workers in arrival order);
* data plane: with the ``nccl`` (RCCL) backend the gradient and the weights move
  GPU-to-GPU over xGMI through a dedicated RCCL group (point-to-point send/recv on
  the server stream); with gloo (CPU plumbing config, or several ranks rehearsing
  on one card) they are staged through host buffers.

Rank 0's own worker talks to the server in-process.  Message tags: GRAD (worker
-> PS, followed by the gradient), DONE (worker -> PS, the done-queue token).

Threads and communicators: on rank 0 only the server thread drives the control
and data groups; on the other ranks only the main thread does.  The trainer's own
collectives during the run (per-epoch evaluation sums, BatchNorm statistics) go
over a third, gloo group on host copies (``dist.set_host_collectives``), so no
rank ever drives two RCCL communicators from two threads without a cross-rank
order (a deadlock pattern); the default group is used again after ``finish()``.
"""

import threading
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..runtime.optim import BETA1, BETA2, EPSILON, adam_reference_, learning_rate

TAG_HDR, TAG_GRAD, TAG_PARAMS = 11, 12, 13
MSG_GRAD, MSG_DONE = 1, 2


class ParameterServer:
    """TF-Adam on the master weights (CPU), applied in gradient arrival order."""

    def __init__(self, flat, cfg):
        self.w = flat.master.detach().to("cpu", torch.float32).clone()
        self.m = flat.m.detach().to("cpu", torch.float32).clone()
        self.v = flat.v.detach().to("cpu", torch.float32).clone()
        self.cfg = cfg
        self.step = flat.global_step
        self.b1p, self.b2p = flat.beta1_power, flat.beta2_power
        self.lock = threading.Lock()
        self.stream = None

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


class DeviceParameterServer(ParameterServer):
    """The server state in rank 0's HBM; one fused native TF-Adam launch per update
    (a single optimizer-only segment: no 16-bit repack), all server work on one
    dedicated stream so concurrent pushes (server thread, rank 0's own worker) are
    ordered on the device exactly as the lock orders them on the host."""

    def __init__(self, flat, cfg):
        from .. import native
        self.C = native.require()
        self.native = native
        dev = flat.master.device
        self.w = flat.master.detach().clone()
        self.m = flat.m.detach().clone()
        self.v = flat.v.detach().clone()
        self.g = torch.zeros_like(self.w)
        self.cfg = cfg
        self.step = flat.global_step
        self.b1p, self.b2p = flat.beta1_power, flat.beta2_power
        self.lock = threading.Lock()
        self.stream = torch.cuda.Stream(device=dev)
        dt = np.dtype([("off", "<i4"), ("n", "<i4"), ("kind", "<i4"), ("T", "<i4"), ("Ci", "<i4"),
                       ("Co", "<i4"), ("Ci_pad", "<i4"), ("rowstride", "<i4"), ("dg_rowstride", "<i4"),
                       ("pad_", "<i4"), ("fwd_off", "<i8"), ("dg_off", "<i8")])
        assert dt.itemsize == self.C.packseg_bytes()
        seg = np.array([(0, self.w.numel(), 0, 0, 0, 0, 0, 0, 0, 0, -1, -1)], dtype=dt)
        self.segs = torch.from_numpy(seg.view(np.uint8).copy()).to(dev)
        self.dummy_arena = torch.zeros(64, dtype=torch.bfloat16, device=dev)

    def apply(self, g: torch.Tensor, out: torch.Tensor) -> int:
        """g: device gradient (ordered on the caller's current stream); out: device
        buffer receiving the weights -- valid on the server stream (callers wait on
        ``self.stream`` before reading it)."""
        with self.lock:
            cur = torch.cuda.current_stream(self.w.device)
            self.stream.wait_stream(cur)
            lr = learning_rate(self.cfg, self.step)
            lr_t = lr * float(np.sqrt(1.0 - self.b2p)) / (1.0 - self.b1p)
            with torch.cuda.stream(self.stream):
                if g.data_ptr() != self.g.data_ptr():
                    self.g.copy_(g, non_blocking=True)
                self.C.adam_pack(self.w.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                 self.w.numel(), self.segs.data_ptr(), 1, lr_t, BETA1, BETA2, EPSILON, 1.0, 1,
                                 self.dummy_arena.data_ptr(), self.native.stream_handle(self.stream))
                out.copy_(self.w, non_blocking=True)
            self.b1p *= BETA1
            self.b2p *= BETA2
            self.step += 1
            return self.step

    def snapshot(self, flat):
        with self.lock:
            self.stream.synchronize()
            flat.master.copy_(self.w)
            flat.m.copy_(self.m)
            flat.v.copy_(self.v)
            flat.global_step = self.step
            flat.beta1_power, flat.beta2_power = self.b1p, self.b2p


class AsyncPS:
    def __init__(self, flat, cfg, ctx, repack=None):
        self.flat = flat
        self.cfg = cfg
        self.ctx = ctx
        self.repack = repack
        self.rank, self.world = ctx.rank, ctx.world_size
        dev = flat.master.device
        self.device = dev
        self.ctrl = dist.new_group(backend="gloo")                 # headers (any-source)
        self.rccl = ctx.backend == "nccl" and dev.type == "cuda"
        self.data = dist.new_group(backend="nccl") if self.rccl else self.ctrl
        # the main thread's collectives while the server runs (module docstring)
        self.coll = dist.new_group(backend="gloo")
        from . import dist as D
        D.set_host_collectives(self.coll)
        self.server: Optional[ParameterServer] = None
        self.thread = None
        # the data-plane buffers: device tensors over RCCL, host buffers over gloo
        bdev = dev if self.rccl else torch.device("cpu")
        self.gbuf = torch.zeros(flat.numel, dtype=torch.float32, device=bdev)
        self.pbuf = torch.zeros(flat.numel + 2, dtype=torch.float32, device=bdev)
        self.ps_step = flat.global_step
        self.local_steps = 0
        if self.rank == 0:
            self.server = DeviceParameterServer(flat, cfg) if dev.type == "cuda" else ParameterServer(flat, cfg)
            self.thread = threading.Thread(target=self._serve, daemon=True)
            self.thread.start()

    # ------------------------------------------------------------- server (rank 0)
    def _serve(self):
        done = 0
        hdr = torch.zeros(2, dtype=torch.int64)
        sv = self.server
        on_dev = isinstance(sv, DeviceParameterServer)
        if on_dev:
            torch.cuda.set_device(self.device)
        bdev = self.device if self.rccl else torch.device("cpu")
        g = torch.zeros(self.flat.numel, dtype=torch.float32, device=bdev)
        w = torch.zeros(self.flat.numel + 2, dtype=torch.float32, device=bdev)
        gd = g if (self.rccl or not on_dev) else torch.zeros(self.flat.numel, dtype=torch.float32, device=self.device)
        wd = w if (self.rccl or not on_dev) else torch.zeros(self.flat.numel + 2, dtype=torch.float32,
                                                            device=self.device)
        ctx = torch.cuda.stream(sv.stream) if on_dev else _Null()
        with ctx:
            while done < self.world - 1:
                src = dist.recv(hdr, src=None, group=self.ctrl, tag=TAG_HDR)
                if int(hdr[0]) == MSG_DONE:
                    done += 1
                    print("Worker #{} reports job finished.".format(src), flush=True)
                    continue
                dist.recv(g, src=src, group=self.data, tag=TAG_GRAD)
                if gd is not g:
                    gd.copy_(g, non_blocking=True)
                step = sv.apply(gd, wd[:-2])
                wd[-2] = float(step & 0xFFFFFF)          # step split in two exact fp32 halves
                wd[-1] = float(step >> 24)
                if wd is not w:
                    w.copy_(wd)                           # host staging (gloo data plane)
                elif on_dev:
                    torch.cuda.current_stream().wait_stream(sv.stream)
                dist.send(w, dst=src, group=self.data, tag=TAG_PARAMS)

    # ------------------------------------------------------------- worker side
    def push_pull(self):
        """Send this worker's gradient, receive the PS weights (one async step)."""
        f = self.flat
        if self.rank == 0:
            sv = self.server
            out = self.pbuf[:-2]
            if isinstance(sv, DeviceParameterServer):
                if getattr(self, "_dev_out", None) is None:
                    self._dev_out = torch.zeros_like(f.master)
                out = self._dev_out
                self.ps_step = sv.apply(f.grad, out)
                torch.cuda.current_stream().wait_stream(sv.stream)
                f.master.copy_(out)
            else:
                self.gbuf.copy_(f.grad)
                self.ps_step = sv.apply(self.gbuf, out)
                f.master.copy_(out.to(f.master.device))
        else:
            hdr = torch.tensor([MSG_GRAD, self.local_steps], dtype=torch.int64)
            dist.send(hdr, dst=0, group=self.ctrl, tag=TAG_HDR)
            if self.rccl:
                dist.send(f.grad, dst=0, group=self.data, tag=TAG_GRAD)
            else:
                self.gbuf.copy_(f.grad)
                dist.send(self.gbuf, dst=0, group=self.data, tag=TAG_GRAD)
            dist.recv(self.pbuf, src=0, group=self.data, tag=TAG_PARAMS)
            tail = self.pbuf[-2:].cpu()
            self.ps_step = int(tail[0].item()) | (int(tail[1].item()) << 24)
            f.master.copy_(self.pbuf[:-2].to(f.master.device, non_blocking=True))
        self.local_steps += 1
        f.global_step = self.ps_step      # the PS's shared global_step, as in TF
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
        if isinstance(sv, DeviceParameterServer):
            sv.snapshot(self.flat)
            return
        with sv.lock:
            dev = self.flat.master.device
            self.flat.master.copy_(sv.w.to(dev))
            self.flat.m.copy_(sv.m.to(dev))
            self.flat.v.copy_(sv.v.to(dev))
            self.flat.global_step = sv.step
            self.flat.beta1_power, self.flat.beta2_power = sv.b1p, sv.b2p

    def finish(self):
        """Done-queue shutdown: workers enqueue a token; the PS waits for all of them."""
        from . import dist as D
        if self.rank != 0:
            hdr = torch.tensor([MSG_DONE, 0], dtype=torch.int64)
            dist.send(hdr, dst=0, group=self.ctrl, tag=TAG_HDR)
        elif self.thread is not None:
            self.thread.join()
            self.snapshot_into_flat()
            if self.repack is not None:
                self.repack()
        D.set_host_collectives(None)       # the server is done: default group again


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
