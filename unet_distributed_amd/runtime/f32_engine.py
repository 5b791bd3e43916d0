"""Native fp32 executor: the reference's own precision on the HIP path.

The reference trains fp32 end to end on CPUs (`test_dist.py:196-202`, TF 1.4 + MKL); the
bf16 / fp16 executor (`native_engine.NativeUNet`) is the fast path.  This one runs the same
training step -- forward, Dice (+ BCE) loss, backward, TF-Adam -- with fp32 storage and
fp32 MFMA (`kernels/f32.hip`, `v_mfma_f32_16x16x4_f32`, exact products), so a user of
the reference gets its numerics on MI355X:

* every activation / gradient buffer is allocated once for the per-GPU batch (NHWC fp32)
  and every launch is recorded once into a native `_C.Plan` and replayed from C++;
* the kernels read the fp32 masters in the TF layouts directly (HWIO conv kernels,
  (kh, kw, Cout, Cin) transposed-conv kernels); the two copies a GEMM needs in another
  layout -- the flipped / transposed data-gradient kernel of each conv and the [Cin][tap
  Cout] forward kernel of each transposed conv -- are refreshed by one transpose launch per
  weight at the start of the step (`f32_transpose`, ~31 MB per step);
* the decoder concat is never materialised (two-source implicit GEMM; its data gradient
  is two launches over the kernel's column ranges), ReLU backward is the consumer's mask
  (`x > 0` of the activation it writes the gradient for), dropout is the same counter hash
  as the bf16 path (`z > 0` of the dropout output is "kept and active"), the max-pool
  backward adds the skip gradient and applies the ReLU mask in one pass;
* weight gradients are split-K slabs reduced in fixed order (deterministic), bias
  gradients fixed-order column sums; TF-Adam is the shared fused launch (`adam.hip`) on
  the flat fp32 master.

The backward plan is cut at allreduce-bucket boundaries like the bf16 executor's, so the
trainer's bucketed RCCL allreduce overlaps it the same way.
"""

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import native
from ..models.spec import UNetSpec
from .params import FlatParams
from .plan_check import RecordingPlan


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


class NativeUNetF32:
    """Plans and runs forward + backward of one fp32 UNet micro-batch on the GPU."""

    WG_SPLIT_TARGET = 256           # split-K slabs per weight gradient (~1 workgroup per CU and tile)

    def __init__(self, spec: UNetSpec, flat: FlatParams, batch: int, img: int, device, loss: str = "dice",
                 bce_weight: float = 1.0, bucket_bounds: Optional[Sequence[int]] = None,
                 eval_dropout: bool = False, dry_run: bool = False):
        self.C = native.require()
        if spec.norm != "none":
            raise NotImplementedError("fp32 native executor: norm=%s (the reference has no normalisation; "
                                      "BatchNorm / GroupNorm run on the bf16 / fp16 executor)" % spec.norm)
        if spec.n_cl_out != 1:
            raise NotImplementedError("fp32 native executor: n_cl_out must be 1")
        self.spec, self.flat = spec, flat
        # dry_run: plan construction only (plan construction itself launches nothing); the
        # static plan validation (runtime/plan_check.py) runs on such an executor on a CPU
        # host, and running its plans is refused
        self._dry = dry_run
        self.B, self.img, self.dims = batch, img, spec.dims
        self.device = torch.device(device)
        self.loss = loss
        self.bce_weight = float(bce_weight) if loss == "dice_bce" else 0.0
        self.dtype = "fp32"
        self.state: Dict[str, torch.Tensor] = {}
        self.fusions: Dict[str, List[str]] = {}
        self.graphs = None
        self.bufs: Dict[str, torch.Tensor] = {}
        self._alloc()
        self.plan = RecordingPlan(self.C.Plan(0))
        self.eval_plan = RecordingPlan(self.C.Plan(0))
        self._layer_done_at: Dict[str, int] = {}
        self._build_forward(self.plan, dropout=True)
        self.fwd_end = self.plan.size()
        self._build_backward(self.plan)
        self.bwd_end = self.plan.size()
        self._build_forward(self.eval_plan, dropout=eval_dropout)
        self.set_buckets(bucket_bounds)
        self._adam_segs()

    # ------------------------------------------------------------------ shapes / buffers
    def sdims(self, level: int):
        s = self.img >> (level - 1)
        return (s, s, s) if self.dims == 3 else (1, s, s)

    def npix(self, level: int) -> int:
        d, h, w = self.sdims(level)
        return self.B * d * h * w

    def _buf(self, name, level, ch):
        d, h, w = self.sdims(level)
        shape = (self.B, h, w, ch) if self.dims == 2 else (self.B, d, h, w, ch)
        t = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.bufs[name] = t
        return t

    def _alloc(self):
        spec = self.spec
        self._buf("x", 1, spec.in_channels)
        self.target = torch.zeros(self.npix(1), dtype=torch.float32, device=self.device)
        self.loss_scale_dev = torch.ones(1, dtype=torch.float32, device=self.device)
        self.tinfo = {"x": (1, spec.in_channels, False, False)}
        self.inputs: Dict[str, tuple] = {}
        cur, pending_up = "x", None
        for l in spec.layers:
            if l.kind == "conv":
                if l.skip_from is not None:
                    src1, up1 = (pending_up, 2) if pending_up is not None else (cur, 1)
                    self.inputs[l.name] = (src1, up1, l.skip_from)
                    pending_up = None
                else:
                    self.inputs[l.name] = (cur, 1, None)
                self._buf(l.name, l.level, l.cout)
                self.tinfo[l.name] = (l.level, l.cout, True, l.dropout and spec.dropout > 0)
                cur = l.name
            elif l.kind == "pool":
                self.inputs[l.name] = (cur, 1, None)
                self._buf(l.name, l.level + 1, l.cout)
                self.tinfo[l.name] = (l.level + 1, l.cout, True, False)
                cur = l.name
            elif l.kind == "tconv":
                self.inputs[l.name] = (cur, 1, None)
                self._buf(l.name, l.level, l.cout)
                self.tinfo[l.name] = (l.level, l.cout, False, False)
                cur = l.name
            elif l.kind == "up":
                pending_up = cur
            elif l.kind == "mask":
                self.inputs[l.name] = (cur, 1, None)
                self.head_in = cur
        hc = self.tinfo[self.head_in][1]
        if hc not in (16, 32, 64):
            raise NotImplementedError("fp32 native executor: head input channels %d" % hc)
        P = self.npix(1)
        self.prob = torch.zeros(P, dtype=torch.float32, device=self.device)
        nb = self.C.f32_head_blocks(P)
        self.head_partial = torch.zeros(nb * (hc + 1) + hc + 1, dtype=torch.float32, device=self.device)
        self.sums = torch.zeros(4, dtype=torch.float32, device=self.device)
        for name in list(self.tinfo):
            if name != "x":
                self.bufs["d:" + name] = torch.zeros_like(self.bufs[name])
        for l in spec.layers:
            if l.kind == "conv" and l.skip_from is not None:
                self.bufs["dskip:" + l.skip_from] = torch.zeros_like(self.bufs[l.skip_from])
                src1, up1, _ = self.inputs[l.name]
                if up1 == 2:
                    d, h, w = self.sdims(l.level)
                    ch = self.tinfo[src1][1]
                    shape = (self.B, h, w, ch) if self.dims == 2 else (self.B, d, h, w, ch)
                    self.bufs["up:" + src1] = torch.zeros(shape, dtype=torch.float32, device=self.device)
                    self.bufs["dfull:" + src1] = torch.zeros(shape, dtype=torch.float32, device=self.device)
        # weight copies in other GEMM layouts (refreshed every step from the masters)
        self.wcopy: Dict[str, torch.Tensor] = {}
        for l in spec.param_layers():
            if l.kind in ("conv", "tconv"):
                n = self.flat.view(self.flat.master, l.name + "/kernel").numel()
                self.wcopy[l.name] = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._colsum_part = torch.zeros(256 * 1024, dtype=torch.float32, device=self.device)

    def master(self, var):
        return _ptr(self.flat.view(self.flat.master, var))

    def grad(self, var):
        return _ptr(self.flat.view(self.flat.grad, var))

    def _salt(self, lname):
        return [l.name for l in self.spec.layers].index(lname)

    def _geo(self, level_out, level_in=None, K=3, stride=1, pad=1):
        od, oh, ow = self.sdims(level_out)
        idd, ih, iw = self.sdims(level_in or level_out)
        kd = K if self.dims == 3 else 1
        return dict(N=self.B, OD=od, OH=oh, OW=ow, ID=idd, IH=ih, IW=iw, KD=kd, KH=K, KW=K, stride=stride, pad=pad)

    # ------------------------------------------------------------------ plans
    def _build_forward(self, plan, dropout):
        spec, b = self.spec, self.bufs
        T2 = 2 ** self.dims
        for l in spec.layers:
            if l.kind == "tconv":
                # forward kernel copy [Cin][tap][Cout] of the (kh, kw, Cout, Cin) master
                plan.add_generic("f32_transpose", [self.master(l.name + "/kernel"), _ptr(self.wcopy[l.name])],
                                 [1, T2 * l.cout, l.cin, 0], [], "pack:" + l.name)
        for l in spec.layers:
            if l.kind == "conv":
                src1, up1, skip = self.inputs[l.name]
                s1 = b[src1]
                if up1 == 2:
                    lvl = self.tinfo[src1][0]
                    dd, hh, ww = self.sdims(lvl)
                    plan.add_generic("f32_ups_fwd", [_ptr(b[src1]), _ptr(b["up:" + src1])],
                                     [self.B, dd, hh, ww, self.tinfo[src1][1], int(self.dims == 3)], [],
                                     "fwd:up:" + src1)
                    s1 = b["up:" + src1]
                d = self._geo(l.level)
                d.update(name="fwd:" + l.name, C1=self.tinfo[src1][1], C2=self.tinfo[skip][1] if skip else 0,
                         src1=_ptr(s1), src2=_ptr(b[skip]) if skip else None, wgt=self.master(l.name + "/kernel"),
                         bias=self.master(l.name + "/bias"), Cout=l.cout, relu=1, dst1=_ptr(b[l.name]),
                         drop_rate=spec.dropout if (l.dropout and dropout) else 0.0, salt=self._salt(l.name))
                plan.add_f32_conv(d)
            elif l.kind == "pool":
                src = self.inputs[l.name][0]
                dd, hh, ww = self.sdims(l.level)
                plan.add_generic("f32_pool_fwd", [_ptr(b[src]), _ptr(b[l.name])],
                                 [self.B, dd, hh, ww, l.cout, int(self.dims == 3)], [], "fwd:" + l.name)
            elif l.kind == "tconv":
                src = self.inputs[l.name][0]
                d = self._geo(l.level + 1, K=1, pad=0)
                d.update(name="fwd:" + l.name, C1=l.cin, src1=_ptr(b[src]), wgt=_ptr(self.wcopy[l.name]),
                         bias=self.master(l.name + "/bias"), Cout=(2 ** self.dims) * l.cout, relu=0,
                         shuffle=self.dims, dst1=_ptr(b[l.name]))
                plan.add_f32_conv(d)
            elif l.kind == "mask":
                hc = self.tinfo[self.head_in][1]
                plan.add_generic("f32_head_fwd", [_ptr(b[self.head_in]), self.master("Mask/kernel"),
                                                  self.master("Mask/bias"), _ptr(self.target), _ptr(self.prob),
                                                  _ptr(self.head_partial), _ptr(self.sums)],
                                 [self.npix(1), hc], [], "fwd:Mask")

    def _mask_of(self, tname):
        """(mask tensor, scale) a data gradient into tensor `tname` applies: the ReLU output
        itself (dropout: z > 0 is kept and active, rescaled by 1 / (1 - rate)); none for
        pool (routed to positive maxima by the pool backward) and linear tconv outputs."""
        lvl, ch, relu, drop = self.tinfo[tname]
        if not relu or tname == "x":
            return None, 1.0
        if self.spec.layers[[l.name for l in self.spec.layers].index(tname)].kind == "pool":
            return None, 1.0
        return self.bufs[tname], (1.0 / (1.0 - self.spec.dropout)) if drop else 1.0

    def _wgrad(self, plan, name, geo, M1, M2, Nc, a1, a2, bsrc, kernel_var, taps, bias_var, bias_src, bias_rows):
        """Weight gradient slabs -> fixed-order reduction into the kernel gradient; bias
        gradient by fixed-order column sums."""
        Q = geo["N"] * geo["QD"] * geo["QH"] * geo["QW"]
        bm, bn = self.C.f32_wgrad_tile(M1, M2, Nc)      # (0, 0): the generic 64 x 64 tile
        bm, bn = bm or 64, bn or 64
        tiles = -(-(M1 + M2) // bm) * -(-Nc // bn) * taps
        splits = max(1, min(self.WG_SPLIT_TARGET // max(1, tiles) * 4, Q // 256, 512))
        slab = torch.empty(splits * taps * (M1 + M2) * Nc, dtype=torch.float32, device=self.device)
        self._keep.append(slab)
        d = dict(geo, name="wgrad:" + name, M1=M1, M2=M2, Nc=Nc, a1=_ptr(a1), a2=_ptr(a2) if a2 is not None else None,
                 b=_ptr(bsrc), slab=_ptr(slab), splits=splits)
        plan.add_f32_wgrad(d)
        stage = torch.empty(max(64, self.C.wgrad_reduce_stage_floats(splits, taps, M1 + M2, Nc)),
                            dtype=torch.float32, device=self.device)
        self._keep.append(stage)
        plan.add_generic("wgrad_reduce", [_ptr(slab), self.grad(kernel_var), _ptr(stage)],
                         [splits, taps, M1 + M2, M1 + M2, Nc], [1.0], "reduce:" + name)
        plan.annotate(reads=[_ptr(slab)], writes=[self.grad(kernel_var)])
        cw = self.flat.view(self.flat.master, bias_var).numel()
        nblk = max(1, min(1024, bias_rows // 2048, self._colsum_part.numel() // cw))
        assert nblk * cw <= self._colsum_part.numel()
        plan.add_generic("f32_colsum", [_ptr(bias_src), _ptr(self._colsum_part), self.grad(bias_var)],
                         [bias_rows, cw, nblk], [], "bsum:" + name)

    def _build_backward(self, plan):
        spec, b = self.spec, self.bufs
        self._keep: List[torch.Tensor] = []
        T3, T2 = 3 ** self.dims, 2 ** self.dims
        # data-gradient kernel copies: [tap'][Cout][Cin] with the taps reversed
        for l in spec.param_layers():
            if l.kind == "conv" and l.name != spec.layers[0].name:
                plan.add_generic("f32_transpose", [self.master(l.name + "/kernel"), _ptr(self.wcopy[l.name])],
                                 [T3, l.cin, l.cout, 1], [], "pack:" + l.name)
        for l in reversed(spec.layers):
            if l.kind == "mask":
                hc = self.tinfo[self.head_in][1]
                plan.add_generic("f32_head_bwd", [_ptr(b[self.head_in]), self.master("Mask/kernel"), _ptr(self.prob),
                                                  _ptr(self.target), _ptr(self.sums), _ptr(b["d:" + self.head_in]),
                                                  _ptr(self.head_partial), self.grad("Mask/kernel"),
                                                  self.grad("Mask/bias")],
                                 [self.npix(1), hc], [1.0 / float(self.npix(1)), self.bce_weight], "bwd:Mask")
                self._layer_done_at["Mask"] = plan.size()
            elif l.kind == "conv":
                src1, up1, skip = self.inputs[l.name]
                first = src1 == "x"
                c1 = self.tinfo[src1][1]
                c2 = self.tinfo[skip][1] if skip else 0
                dy = b["d:" + l.name]
                a1 = b["up:" + src1] if up1 == 2 else b[src1]
                od, oh, ow = self.sdims(l.level)
                geo = dict(N=self.B, QD=od, QH=oh, QW=ow, AD=od, AH=oh, AW=ow, KD=3 if self.dims == 3 else 1,
                           KH=3, KW=3, stride=1, pad=1)
                self._wgrad(plan, l.name, geo, c1, c2, l.cout, a1, b[skip] if skip else None, dy,
                            l.name + "/kernel", T3, l.name + "/bias", dy, self.npix(l.level))
                if not first:
                    # data gradient: conv of dY with the flipped, transposed kernel; the
                    # concat input's halves are two launches over its column ranges
                    parts = [(0, c1, "dfull:" + src1 if up1 == 2 else "d:" + src1, src1 if up1 == 1 else None)]
                    if skip:
                        parts.append((c1, c2, "dskip:" + skip, None))
                    for off, cc, dst, mtensor in parts:
                        mk, ms = self._mask_of(mtensor) if mtensor else (None, 1.0)
                        d = self._geo(l.level)
                        d.update(name="dgrad:" + l.name, C1=l.cout, src1=_ptr(dy),
                                 wgt=_ptr(self.wcopy[l.name]) + 4 * off, ldw=c1 + c2, Cout=cc, relu=0,
                                 dst1=_ptr(b[dst]), mask1=_ptr(mk) if mk is not None else None, mask_scale1=ms)
                        plan.add_f32_conv(d)
                    if up1 == 2:
                        lvl = self.tinfo[src1][0]
                        dd, hh, ww = self.sdims(lvl)
                        mk, _ = self._mask_of(src1)
                        plan.add_generic("f32_ups_bwd", [_ptr(b["dfull:" + src1]), _ptr(mk), _ptr(b["d:" + src1])],
                                         [self.B, dd, hh, ww, c1, int(self.dims == 3)], [], "bwd:up:" + src1)
                self._layer_done_at[l.name] = plan.size()
            elif l.kind == "pool":
                src = self.inputs[l.name][0]
                dd, hh, ww = self.sdims(l.level)
                sk = b.get("dskip:" + src)
                plan.add_generic("f32_pool_bwd", [_ptr(b[src]), _ptr(b["d:" + l.name]), _ptr(sk), _ptr(b["d:" + src])],
                                 [self.B, dd, hh, ww, l.cout, int(self.dims == 3)], [], "bwd:" + l.name)
            elif l.kind == "tconv":
                src = self.inputs[l.name][0]
                du = b["d:" + l.name]
                lo, hi = self.sdims(l.level + 1), self.sdims(l.level)
                geo = dict(N=self.B, QD=lo[0], QH=lo[1], QW=lo[2], AD=hi[0], AH=hi[1], AW=hi[2],
                           KD=2 if self.dims == 3 else 1, KH=2, KW=2, stride=2, pad=0)
                self._wgrad(plan, l.name, geo, l.cout, 0, l.cin, du, None, b[src], l.name + "/kernel", T2,
                            l.name + "/bias", du, self.npix(l.level))
                mk, ms = self._mask_of(src)
                d = self._geo(l.level + 1, l.level, K=2, stride=2, pad=0)
                d.update(name="dgrad:" + l.name, C1=l.cout, src1=_ptr(du), wgt=self.master(l.name + "/kernel"),
                         Cout=l.cin, relu=0, dst1=_ptr(b["d:" + src]), mask1=_ptr(mk) if mk is not None else None,
                         mask_scale1=ms)
                plan.add_f32_conv(d)
                self._layer_done_at[l.name] = plan.size()

    # ------------------------------------------------------------------ buckets / Adam
    def set_buckets(self, bounds: Optional[Sequence[int]]):
        self.seg_ends = []
        if not bounds:
            self.seg_ends = [self.bwd_end]
            return
        for bound in bounds:
            last = self.fwd_end
            for name, shape, off, n in self.flat.entries:
                if off < bound:
                    last = max(last, self._layer_done_at[name.split("/")[0]])
            self.seg_ends.append(last)
        self.seg_ends[-1] = self.bwd_end

    def _adam_segs(self):
        """Adam over the whole flat buffer, no 16-bit repack (kind-0 segments)."""
        f = self.flat
        dt = np.dtype([("off", "<i4"), ("n", "<i4"), ("kind", "<i4"), ("T", "<i4"), ("Ci", "<i4"),
                       ("Co", "<i4"), ("Ci_pad", "<i4"), ("rowstride", "<i4"), ("dg_rowstride", "<i4"),
                       ("pad_", "<i4"), ("fwd_off", "<i8"), ("dg_off", "<i8")])
        ends = [e[2] for e in f.entries[1:]] + [f.numel]
        segs = [(off, end - off, 0, 0, 0, 0, 0, 0, 0, 0, -1, -1) for (_, _, off, _), end in zip(f.entries, ends)]
        arr = np.array(segs, dtype=dt)
        assert dt.itemsize == self.C.packseg_bytes()
        self.nseg = len(segs)
        self.segs = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)

    def repack(self, stream=None):
        """(no 16-bit copies: the per-step weight layouts are refreshed inside the plans)"""

    def adam_step(self, lr, beta1_power, beta2_power, grad_scale=1.0, stream=None, beta1=0.9, beta2=0.999,
                  eps=1e-8):
        f = self.flat
        lr_t = lr * math.sqrt(1.0 - beta2_power) / (1.0 - beta1_power)
        self.C.adam_pack(_ptr(f.master), _ptr(f.grad), _ptr(f.m), _ptr(f.v), f.numel, _ptr(self.segs), self.nseg,
                         lr_t, beta1, beta2, eps, grad_scale, 1, 0, native.stream_handle(stream), dtype=0)

    # ------------------------------------------------------------------ running
    def enable_graphs(self):
        """(eager replay of the native plan: the fp32 step is GEMM-bound, launch gaps are noise)"""

    def set_loss_scale(self, scale: float):
        if scale != 1.0:
            raise NotImplementedError("fp32 executor: no loss scaling")

    def load_batch(self, x: torch.Tensor, y: torch.Tensor, stream=None):
        self.bufs["x"].view(-1).copy_(x.reshape(-1), non_blocking=True)
        self.target.copy_(y.reshape(-1), non_blocking=True)

    def load_indexed(self, x_all, y_all, idx, stream=None):
        self.bufs["x"].copy_(x_all.index_select(0, idx).view_as(self.bufs["x"]))
        self.target.copy_(y_all.index_select(0, idx).reshape(-1))

    def _live(self):
        if self._dry:
            raise RuntimeError("fp32 executor built with dry_run=True: its plans are for validation only")

    def forward(self, seed: int, stream=None):
        self._live()
        self.plan.set_seed(seed & 0xFFFFFFFF)
        self.plan.run(0, self.fwd_end, native.stream_handle(stream))

    def backward(self, on_segment=None, stream=None):
        self._live()
        s = native.stream_handle(stream)
        begin = self.fwd_end
        for i, end in enumerate(self.seg_ends):
            if end > begin:
                self.plan.run(begin, end, s)
            begin = max(begin, end)
            if on_segment is not None:
                on_segment(i)

    def evaluate_batch(self, stream=None):
        self._live()
        self.eval_plan.set_seed(0)
        self.eval_plan.run(0, self.eval_plan.size(), native.stream_handle(stream))

    def probs(self) -> torch.Tensor:
        d, h, w = self.sdims(1)
        shape = (self.B, h, w, 1) if self.dims == 2 else (self.B, d, h, w, 1)
        return self.prob.view(shape)
