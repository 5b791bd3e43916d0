"""Step backends: one forward + backward of the local micro-batch into the flat
gradient buffer.

* ``NativeBackend`` -- the MI355X path: the planned HIP executor
  (``runtime.native_engine.NativeUNet``).  Mandatory on GPU for the configs
  it supports; never silently replaced by ATen.
* ``TorchBackend`` -- ATen reference (CPU plumbing config, fp32 runs, and the
  numerical oracle for the kernels).

Both expose ``fwd_bwd(x, y, seed, on_segment)``, ``sums()`` (device tensor
{I, St, Sp, BCE_sum} of the last forward) and ``eval_sums(x, y)``.
"""

from typing import Callable, Optional

import torch

from ..models import reference
from ..ops import losses
from .params import FlatParams


class TorchBackend:
    name = "torch"

    def __init__(self, spec, flat: FlatParams, cfg, device, per_rank_batch: int, bounds=None):
        self.spec = spec
        self.flat = flat
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[cfg.dtype]
        if self.device.type == "cpu" and self.dtype == torch.float16:
            self.dtype = torch.float32
        self._sums = torch.zeros(4, device=self.device)
        self.state = {}
        if spec.norm == "batch":
            for l in spec.param_layers():
                if l.kind == "conv":
                    self.state[l.name + "/norm/moving_mean"] = torch.zeros(l.cout, device=self.device)
                    self.state[l.name + "/norm/moving_variance"] = torch.ones(l.cout, device=self.device)
        # allreduce buckets: on_segment(k) is called once per bucket after the backward
        # (the GradSync of the trainer is planned with the same bounds)
        self.bounds = list(bounds) if bounds else [flat.numel]

    def set_buckets(self, bounds):
        self.bounds = list(bounds)

    def _forward_logits(self, params, x, train, seed, dropout):
        with torch.autocast(self.device.type, dtype=self.dtype, enabled=self.dtype != torch.float32):
            return reference.forward(self.spec, params, x.to(self.device), train=train, dropout=dropout,
                                     seed=seed, state=self.state, return_logits=True)

    def fwd_bwd(self, x, y, seed: int, on_segment: Optional[Callable[[int], None]] = None,
                grad_scale: float = 1.0):
        if hasattr(x, "x_all"):
            x, y = x.tensors()
        names = [e[0] for e in self.flat.entries]
        leaves = {n: self.flat.view(self.flat.master, n).detach().requires_grad_(True) for n in names}
        logits = self._forward_logits(leaves, x, True, seed, True).float()
        t = y.to(self.device).float()
        loss, p = losses.total_loss(t, logits, self.cfg.loss, self.cfg.bce_weight)
        grads = torch.autograd.grad(loss * grad_scale, [leaves[n] for n in names], allow_unused=True)
        for n, g in zip(names, grads):
            gv = self.flat.view(self.flat.grad, n)
            if g is None:
                gv.zero_()
            else:
                gv.copy_(g)
        with torch.no_grad():
            i, st, sp = losses.dice_sums(t, p)
            bce = torch.nn.functional.binary_cross_entropy_with_logits(logits, t, reduction="sum")
            self._sums = torch.stack([i, st, sp, bce]).detach()
        self._last = (x, t, p.detach())
        if on_segment is not None:
            for k in range(len(self.bounds)):
                on_segment(k)

    def sums(self) -> torch.Tensor:
        return self._sums

    def summary_images(self, n: int) -> dict:
        """First n samples of the last training batch (channel 0; 3D: middle slice)."""
        x, t, p = self._last
        return _summary_arrays(x, t, p, n)

    @torch.no_grad()
    def eval_sums(self, x, y) -> torch.Tensor:
        logits = self._forward_logits(self.flat.params(), x, False, 0, self.cfg.eval_dropout).float()
        t = y.to(self.device).float()
        p = torch.sigmoid(logits)
        i, st, sp = losses.dice_sums(t, p)
        bce = torch.nn.functional.binary_cross_entropy_with_logits(logits, t, reduction="sum")
        return torch.stack([i, st, sp, bce])

    @torch.no_grad()
    def predict(self, x) -> torch.Tensor:
        logits = self._forward_logits(self.flat.params(), x, False, 0, self.cfg.eval_dropout).float()
        return torch.sigmoid(logits)

    def after_optimizer(self):
        pass


class NativeBackend:
    name = "native"

    def __init__(self, spec, flat: FlatParams, cfg, device, per_rank_batch: int, bounds=None):
        from .native_engine import NativeUNet
        from .f32_engine import NativeUNetF32
        self.cfg = cfg
        self.flat = flat
        if cfg.dtype == "fp32":
            # the reference's precision (test_dist.py:196-202): fp32 storage, fp32 MFMA
            self.engine = NativeUNetF32(spec, flat, per_rank_batch, cfg.img_size, device, loss=cfg.loss,
                                        bce_weight=cfg.bce_weight, bucket_bounds=bounds,
                                        eval_dropout=cfg.eval_dropout)
        else:
            self.engine = NativeUNet(spec, flat, per_rank_batch, cfg.img_size, device, loss=cfg.loss,
                                     bce_weight=cfg.bce_weight, bucket_bounds=bounds,
                                     eval_dropout=cfg.eval_dropout, dtype=cfg.dtype)
        self.B = per_rank_batch
        if getattr(cfg, "hip_graph", False):
            self.engine.enable_graphs()
        self.state = self.engine.state        # BatchNorm running statistics (checkpointed)

    def set_buckets(self, bounds):
        self.engine.set_buckets(bounds)

    def fwd_bwd(self, x, y, seed: int, on_segment=None, grad_scale: float = 1.0):
        """x, y: batch tensors, or x = a data.loader.ResidentBatch (y unused)."""
        e = self.engine
        e.set_loss_scale(grad_scale)
        if hasattr(x, "x_all"):
            e.load_indexed(x.x_all, x.y_all, x.idx)
        else:
            e.load_batch(x, y)
        e.forward(seed)
        e.backward(on_segment)

    def sums(self) -> torch.Tensor:
        return self.engine.sums

    def summary_images(self, n: int) -> dict:
        """From the buffers the step already holds (no extra forward, Q8): the padded
        16-bit input, the target and the head's probabilities."""
        e = self.engine
        d, h, w = e.sdims(1)
        shape = (e.B, h, w) if e.dims == 2 else (e.B, d, h, w)
        x = e.bufs["x"][..., 0]
        return _summary_arrays(x, e.target.view(shape), e.prob.view(shape), n)

    @torch.no_grad()
    def eval_sums(self, x, y) -> torch.Tensor:
        e = self.engine
        if x.shape[0] != e.B:
            raise ValueError("native eval batch must equal the per-rank batch")
        e.load_batch(x, y)
        e.evaluate_batch()
        return e.sums.clone()

    @torch.no_grad()
    def predict(self, x) -> torch.Tensor:
        e = self.engine
        e.load_batch(x, torch.zeros(x.shape[:-1] + (1,), device=x.device))
        e.evaluate_batch()
        return e.probs().clone()

    def adam_step(self, lr, b1p, b2p, grad_scale=1.0):
        self.engine.adam_step(lr, b1p, b2p, grad_scale)


def _summary_arrays(x, t, p, n) -> dict:
    def prep(a):
        a = a[:n].detach().float()
        if a.dim() == 5:                     # [n, D, H, W, 1]
            a = a[..., 0]
        if a.dim() == 4 and a.shape[-1] == 1:
            a = a[..., 0]
        if a.dim() == 4:                     # 3D volume [n, D, H, W]: middle slice
            a = a[:, a.shape[1] // 2]
        return a.cpu().numpy()
    if x.dim() == 4 and x.shape[-1] > 1 and t.dim() == 4 and t.shape[-1] == 1:
        x = x[..., 0]                        # NHWC input: first channel
    elif x.dim() == 5 and x.shape[-1] > 1:
        x = x[..., 0]
    return {"predictions": prep(p), "ground_truth": prep(t), "images": prep(x)}


def native_supported(spec, cfg, device) -> Optional[str]:
    """None if the native executor supports this config, else the reason."""
    if torch.device(device).type != "cuda":
        return "not on a GPU"
    if cfg.dtype not in ("bf16", "fp16", "fp32"):
        return "native kernels are bf16 / fp16 / fp32 (dtype=%s)" % cfg.dtype
    if spec.n_cl_out != 1:
        return "n_cl_out != 1"
    if cfg.dtype == "fp32":
        # (runtime/f32_engine.py: the reference's own configuration family)
        if spec.norm != "none":
            return "the fp32 executor runs the reference's norm-free model (norm=%s: use bf16 / fp16)" % spec.norm
        if spec.base not in (16, 32, 64):
            return "fp32 head input channels must be 16, 32 or 64 (base %d)" % spec.base
        return None
    if spec.base not in (32, 64):
        # the fused head / head kernels take 16, 32 or 64 head-input channels and the
        # row-window kernels 32-channel chunks
        return "base filters must be 32 or 64 (got %d)" % spec.base
    cin = spec.in_channels
    if not (cin <= 8 or cin % 32 == 0):
        return "in_channels=%d" % cin
    return None


def resolve_backend(want: str, spec, cfg, device) -> str:
    """'native' or 'torch' for a requested ``--backend`` (auto / native / torch).

    One GPU path: on a GPU, ``auto`` means the HIP executor and a
    config it does not support is an error with the reason -- never a silent ATen /
    MIOpen run.  ATen stays reachable only by asking for it (``--backend torch``: the
    numerical oracle and baseline) and is what ``auto`` means off the GPU (the CPU /
    gloo plumbing config)."""
    if want == "torch":
        return "torch"
    reason = native_supported(spec, cfg, device)
    on_gpu = torch.device(device).type == "cuda"
    if want == "native" or (want == "auto" and on_gpu):
        if reason is not None:
            raise RuntimeError("the native HIP executor does not support this config (%s); "
                               "pass --backend torch to run the ATen reference path explicitly" % reason)
        return "native"
    return "torch"


def make_backend(spec, flat, cfg, device, per_rank_batch, bounds=None):
    if resolve_backend(cfg.backend, spec, cfg, device) == "native":
        from .. import native
        native.require()
        return NativeBackend(spec, flat, cfg, device, per_rank_batch, bounds)
    return TorchBackend(spec, flat, cfg, device, per_rank_batch, bounds)
