"""Native (HIP/gfx950) static-graph executor for the UNet training step.

The executor plays the role of the reference's TF graph + session
(`test_dist.py:183-298` graph construction, `test_dist.py:396-398` one
``sess.run`` per step), designed for MI355X:

* every activation / gradient buffer of the step is allocated ONCE for the
  per-GPU micro-batch (channels-last bf16, sized for 288 GB HBM3E) and
  reused every step — no allocator traffic in the hot loop;
* every kernel launch of forward + backward is recorded once into a native
  ``_C.Plan`` (shapes, pointers, epilogue flags resolved at plan time) and
  replayed from C++;
* cross-layer fusions that autograd cannot express are planned here:
  - ReLU backward is folded into the CONSUMER's dgrad epilogue (every tensor
    produced by a ReLU is masked by ``x > 0`` by whoever reads it), and the
    dropout keep-mask needs no storage: ``z > 0`` of the dropout output is
    exactly "kept and active", the 1/(1-rate) rescale rides on the same
    epilogue (`model.py:60,66`);
  - the decoder skip concat is never materialised: conv{j}a reads two
    sources in its K loop, its dgrad writes two destinations and the skip
    half is added to the max-pool backward in one kernel;
  - nearest upsampling is folded into the next conv's address generation;
  - bias gradients are column sums fused into the weight-gradient kernel;
  - the Mask 1x1 conv + sigmoid + Dice/BCE partial sums is one kernel.
* the backward plan is split into segments at allreduce-bucket boundaries so
  the trainer can start RCCL allreduces of finished buckets on a side stream
  while later layers' backward still runs.
"""

import math
import os
from contextlib import nullcontext as _nullctx
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native
from ..models.spec import UNetSpec
from .params import FlatParams
from .plan_check import RecordingPlan



def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


def _r64(k: int) -> int:
    return (k + 63) // 64 * 64


# Executor options, each fixed at its measured default (profiles/r*_bench_history.md);
# UNET_ENGINE="key=value,..." overrides them for same-box A/B runs, and tests pass
# ``opts`` to NativeUNet directly.  The only environment variable the executor reads.
#   dual_stream  weight-gradient launches on a side stream during the backward (1)
#   fwd_streams  training forward as two half-batch chunks on two streams (2)
#   head_fuse    Mask head in the epilogue of its input conv's forward (1)
#   head_onload  the head input's gradient formed on load by its consumers (1: 2D; 2: 3D too)
#   head_wsum    the Mask gradients from per-workgroup sums of the fused-head forward; the head
#                input is not stored (1)
#   skip_onload  normalised configs: conv9a's skip source read as pre-norm z by its consumers, never
#                stored in training (1)
#   win_cp3      win_cp of the 3D model (2: the 3D level-1 convs on the chunk-pipelined 128-wide
#                window, conv_win_cp128_kernel -- -10..-12 % per launch, +2 % on the 3D step in
#                round 6; neutral in round 5, before the 3D weight-gradient prefetch)
#   wg_pf        128-wide window weight gradients with the next window's rows + dY prefetched in
#                registers (conv_wgrad.hip wgrad_pf128_kernel): 1 = 3D, 2 = 2D as well (1: the 3D
#                level-1 weight gradients -19..-21 % per launch; 2D neutral)
#   xf_drop      dropout layers' outputs normalised on load too (xform 1 with xd_*) (0: measured
#                slower -- the per-element hash on the consumer's chunk path, r6_bench_history.md)
#   tconv_fused  deepest fine level whose transposed conv runs the composite backward (2; 0 off)
#   tconv_wa     the consumer conv's u-row weight gradient from the composite backward's
#                slab sums (1; 0: full weight gradient over u)
#   tconv_onload deepest fine level whose transposed-conv output u is formed on load by its
#                consumer's forward where nothing else reads it (1; 0: materialised)
#   fwd_offset   layers of chunk 0 before the second forward chunk starts (6)
#   wg_target    weight-gradient split-K grid target, workgroups per gradient (512)
#   dw_fuse      data + weight gradient of a 32 -> 32 channel conv on 128-wide rows in one kernel
#                reading dY once (conv_dw.hip) (1)
#   dw_wgs       workgroups (= slab rows) per fused data + weight gradient launch (512)
#   win_pf       windows per workgroup of the persistent prefetching row window on 128-wide
#                32 -> 32 channel convs (conv_win.h conv_win_pf_kernel) (8; 0 off)
#   win_cp       64-channel row windows on 64-wide rows load the next input chunk under the
#                current chunk's MFMAs (conv_win.h conv_win_cp_kernel) (1; 0 off)
#   dz_split     normalised layers on 16..64-wide rows whose dz only their own data and weight
#                gradients read: both form it on load (conv_win.h XF 2, wgrad_win_kernel DZ) (0:
#                measured slower, r6_bench_history.md -- the consumers' per-window z loads and
#                transform cost more than the norm_bwd_apply pass they replace)
#   wg_pair      row-window weight gradients of 32-channel output blocks with wave-pair partials
#                (conv_wgrad.hip wgrad_win_kernel PAIR: three workgroups per CU): 1 = 3D only,
#                2 = 2D as well, 0 off (0)
#   head_wsum    Mask weight gradients from the fused-head forward's sums: 1 = 2D (with head-on-load),
#                2 = 3D as well (head_dy forms dY from the ReLU bits; measured neutral on 3D b8), 0 off (1)
#   tail3        3D: the last data gradient in two volume halves (tail_halves) (0: measured neutral)
#   route3       3D: the decoder's skip-half data gradient carries the pool backward in its
#                epilogue (skip_route; the data gradient splits in two launches) (1: measured
#                -0.26 ms launch sum, +1.5..3 % 3D b8 bench, r6_bench_history.md)
ENGINE_DEFAULTS = dict(dual_stream=1, fwd_streams=2, head_fuse=1, head_onload=1, tconv_fused=2, tconv_wa=1,
                       tconv_onload=1, fwd_offset=6, wg_target=512, dw_fuse=1, dw_wgs=512, win_pf=8, win_cp=1,
                       wg_pair=0, dz_split=0, head_wsum=1, xf_drop=0, wg_pf=1, win_cp3=2, skip_onload=1,
                       route3=1, tail3=0)


class Fusion:
    """Declarative precondition of one planner fusion: the config-level conditions under
    which the planner may apply it.  Each decision site first asks ``_fusion_ok(name)``;
    only per-layer structure (channel multiples, a single consumer, ...) and the kernel
    probe (``conv_fwd_grid``) stay at the site.  `needs`: fusions that must be active for
    the same layer (a tconv on load reads nothing but what the chained weight gradient
    leaves unread).  tests/test_plan_check.py enumerates norm x decoder x dims x img and
    validates every plan statically (runtime/plan_check.py)."""

    def __init__(self, doc, norm=None, dims=None, decoder=None, img=None, option=None, needs=(),
                 even_batch=False, cpad=None, when=None):
        self.doc, self.norm, self.dims, self.decoder, self.img = doc, norm, dims, decoder, img
        self.option, self.needs, self.even_batch, self.cpad, self.when = option, tuple(needs), even_batch, cpad, when

    def unmet(self, e) -> List[str]:
        """Conditions this config violates (empty: the fusion may apply)."""
        out = []
        if self.norm is not None and e.spec.norm not in self.norm:
            out.append("norm=%s" % e.spec.norm)
        if self.dims is not None and e.dims not in self.dims:
            out.append("dims=%d" % e.dims)
        dec = "upsampling" if e.spec.use_upsampling else "transposed"
        if self.decoder is not None and dec not in self.decoder:
            out.append("decoder=%s" % dec)
        if self.img is not None and e.img not in self.img:
            out.append("img=%d" % e.img)
        if self.option is not None and not e.opts[self.option]:
            out.append("option %s=0" % self.option)
        if self.even_batch and e.B % 2:
            out.append("odd batch")
        if self.cpad is not None and e.cpad not in self.cpad:
            out.append("padded input channels %d" % e.cpad)
        if self.when is not None and not self.when(e):
            out.append("structure")
        return out


_ROW_IMGS = (16, 32, 64, 128)       # 2D images whose rows the row-window kernels take whole
FUSIONS: Dict[str, Fusion] = {
    "head_onload": Fusion("head input gradient formed on load by its consumers (head_grad.h)",
                          norm={"none"}, img=_ROW_IMGS, option="head_onload",
                          when=lambda e: e.tinfo[e.head_in][1] == 32 and e.wgrad_win >= 0 and
                          (e.dims == 2 or (e.img >= 32 and e.opts["head_onload"] >= 2))),
                          # (3D: opt-in, the column-unit window wgrad; measured 0.6 ms slower at b8 --
                          # the 3D weight gradient re-forms each depth tap's head gradient)
    "head_fuse": Fusion("Mask head in the epilogue of its input conv's forward",
                        norm={"none"}, option="head_fuse", when=lambda e: e.tinfo[e.head_in][1] == 32),
    "head_wsum": Fusion("Mask weight / bias gradients from sums the head-input conv's forward accumulates "
                        "(conv_params.h head_ws): the head input is never stored -- 2D: with head-on-load, no "
                        "backward pass over it; 3D (option head_wsum=2): its dY from the ReLU bits (head_dy)",
                        norm={"none"}, option="head_wsum", needs=("head_fuse",),
                        when=lambda e: (e.dims == 2 and e.head_onload) or (e.dims == 3 and e.opts["head_wsum"] >= 2)),
    "pool_epilogue": Fusion("2x2 max-pool in the convNb forward epilogue", norm={"none"}),
    "fwd_2streams": Fusion("training forward as two half-batch chunks on two streams",
                           norm={"none", "group"}, even_batch=True, when=lambda e: e.opts["fwd_streams"] == 2),
    "tconv_fused": Fusion("composite transposed-conv backward (tconv_fused.hip)", dims={2},
                          option="tconv_fused"),
    "tconv_wa": Fusion("consumer's u-row weight gradient chained from the slab sums", dims={2},
                       option="tconv_wa", needs=("tconv_fused",)),
    "tconv_onload": Fusion("transposed conv formed on load by its consumer's forward (XF 5)", dims={2},
                           option="tconv_onload", needs=("tconv_wa",)),
    "skip_onload": Fusion("a normalised skip source normalised on load by its tconv-on-load consumer and the "
                          "chained skip-row weight gradient: never stored in training (x2a / xform 1)",
                          norm={"batch", "group"}, dims={2}, option="skip_onload", when=lambda e: e.wgrad_win >= 0),
    "norm_onload": Fusion("normalisation of an 'a' conv's output on load by its consumer (XF 1)",
                          norm={"batch", "group"}, dims={2}),
    "skip_route": Fusion("skip-half data gradient with the pool backward in its epilogue",
                         when=lambda e: e.dims == 2 or e.opts["route3"] >= 1),
    "tail_halves": Fusion("last data gradient in two batch halves (first-layer wgrad overlap)",
                          norm={"none"}, img=_ROW_IMGS, even_batch=True, cpad=(4, 8),
                          when=lambda e: e.wgrad_win >= 0 and (e.dims == 2 or e.opts["tail3"] >= 1)),
    "dw_fused": Fusion("data + weight gradient from one staged dY halo (conv_dw.hip; 128-pixel segments of "
                       "wider rows)", dims={2}, img=(128, 256, 512, 1024), option="dw_fuse",
                       when=lambda e: e.wgrad_win >= 0),
    "dz_onload": Fusion("norm backward dz = ca g + cb z + cc formed in the fused data + weight gradient's "
                        "halo (conv_dw.hip XF 2): no norm_bwd_apply pass, dz never stored",
                        norm={"batch", "group"}, dims={2}, img=(128,), option="dw_fuse", needs=("dw_fused",)),
    "dz_split": Fusion("norm backward dz formed on load by both of the layer's split consumers -- the "
                       "row-window data gradient (conv_win.h XF 2 / chunk-pipelined DZ) and the window weight "
                       "gradient's B operand (wgrad_win_kernel DZ): no norm_bwd_apply pass, dz never stored",
                       norm={"batch", "group"}, dims={2}, option="dz_split", when=lambda e: e.wgrad_win >= 0),
    "first_dz_onload": Fusion("first layer's norm-backward dz formed by its window wgrad (XF 2)",
                              norm={"batch", "group"}, dims={2}, img=_ROW_IMGS, cpad=(4, 8),
                              when=lambda e: e.wgrad_win >= 0),
}


def engine_options(overrides: Optional[Dict[str, int]] = None) -> Dict[str, int]:
    opts = dict(ENGINE_DEFAULTS)
    for kv in filter(None, os.environ.get("UNET_ENGINE", "").split(",")):
        k, v = kv.split("=")
        if k.strip() not in opts:
            raise ValueError("UNET_ENGINE: unknown option %r (known: %s)" % (k, ", ".join(opts)))
        opts[k.strip()] = int(v)
    for k, v in (overrides or {}).items():
        if k not in opts:
            raise ValueError("engine option %r unknown (known: %s)" % (k, ", ".join(opts)))
        opts[k] = int(v)
    if opts["tconv_fused"] not in (0, 1, 2):
        raise ValueError("tconv_fused must be 0..2 (level 3 measured -2.4 %% / +0.2 %%: removed)")
    return opts


class NativeUNet:
    """Plans and runs forward + backward of one UNet micro-batch on the GPU."""

    def __init__(self, spec: UNetSpec, flat: FlatParams, batch: int, img: int,
                 device, loss: str = "dice", bce_weight: float = 1.0,
                 bucket_bounds: Optional[Sequence[int]] = None, eval_dropout: bool = False,
                 dry_run: bool = False, dtype: str = "bf16", opts: Optional[Dict[str, int]] = None):
        self.C = native.require()
        self.opts = engine_options(opts)
        if spec.norm not in ("none", "batch", "group"):
            raise NotImplementedError("native executor: norm=%s" % spec.norm)
        if spec.n_cl_out != 1:
            raise NotImplementedError("native executor: n_cl_out must be 1")
        self.spec = spec
        self.flat = flat
        self.graphs = None      # HIP-graph cache (enable_graphs)
        # Weight-gradient launches (wgrad / bias colsum / split-K reduce) are off the
        # backward critical path (the dgrad chain): run them on a side stream so they
        # overlap the memory-bound dgrads (option dual_stream=0 disables; measured
        # 5.09 -> 4.83 ms per backward at b256, scripts/dual_stream_probe.py).  HIP graph
        # replay serialises parallel branches on this stack, so the dual-stream
        # backward is launched eagerly even in HIP-graph mode.
        self.dual_stream = bool(self.opts["dual_stream"])
        self._side = None
        self._groups: Dict[tuple, list] = {}
        # 16-bit element type of activations, gradients w.r.t. activations and the
        # weight copies: selects the bf16 or fp16 build of every kernel (common.h)
        if dtype not in ("bf16", "fp16"):
            raise NotImplementedError("native executor: dtype=%s" % dtype)
        self.dtype = dtype
        self.adt = torch.bfloat16 if dtype == "bf16" else torch.float16
        self.dt_id = 0 if dtype == "bf16" else 1
        self.B = batch
        self.img = img
        self.dims = spec.dims
        self.device = torch.device(device)
        self.loss = loss
        self.bce_weight = float(bce_weight) if loss == "dice_bce" else 0.0
        cin = spec.in_channels
        if cin <= 4:
            self.cpad = 4
        elif cin <= 8:
            self.cpad = 8
        elif cin % 32 == 0:
            self.cpad = cin
        else:
            raise NotImplementedError("native executor: in_channels=%d" % cin)
        self.bufs: Dict[str, torch.Tensor] = {}
        # wgrad split-K grid target (workgroups per weight gradient): ~2 per CU.  Dual
        # stream at the default per-GPU batch 1024: 512 > 768 > 384 > 256 > 1024 >> 128
        # (same-box sweep, +1.7 % over 256; 640 re-measured -0.4 % at the round-2 end)
        self.wg_target = self.opts["wg_target"]
        # row-window convs walk their windows in the reverse of the order their input was
        # written (bit 0 forward, bit 1 data gradients; see _rev_order)
        self._rev_mode = 3
        # -1: never use the row-window weight-gradient kernel (set by A/B tests)
        self.wgrad_win = 0
        # fusion name -> layers it was applied to (FUSIONS; plan validation and tests)
        self.fusions: Dict[str, List[str]] = {}
        self._dry = dry_run
        self._alloc_weights()
        self._alloc_activations()
        # (each op's parameters are kept for the static plan validation, runtime/plan_check.py)
        self.plan = RecordingPlan(self.C.Plan(self.dt_id), self._stat_rows_of)
        self.eval_plan = RecordingPlan(self.C.Plan(self.dt_id), self._stat_rows_of)
        for cname, d in self._ut_probe.items():
            self._plan_skip_onload(next(x for x in self.spec.layers if x.name == cname), d)
        self._plan_xforms()
        self._norm_head_loss = False
        self._build_forward(self.plan, dropout=True)
        self.fwd_end = self.plan.size()
        self.seg_ends: List[int] = []
        self._layer_done_at: Dict[str, int] = {}
        self._build_backward(self.plan)
        self.bwd_end = self.plan.size()
        self._build_forward(self.eval_plan, dropout=eval_dropout, train=False)
        self.set_buckets(bucket_bounds)
        if not dry_run:          # dry_run: plan construction only (CPU tests, no GPU launches)
            self.repack()

    def _stat_rows_of(self, d):
        """Statistics rows a conv launch writes (plan validation of the stats extents)."""
        try:
            return self.C.conv_stat_tiles(dict(d, stats=1))[0]
        except ValueError:
            return 0

    # ------------------------------------------------------------------ fusion preconditions
    def _fusion_ok(self, name: str, layer: Optional[str] = None) -> bool:
        """Config-level preconditions of fusion `name` (FUSIONS) hold, and for a per-layer
        fusion every fusion it needs is active for `layer`."""
        f = FUSIONS[name]
        if f.unmet(self):
            return False
        return all(layer in self.fusions.get(n, ()) for n in f.needs) if layer is not None else \
            all(self.fusions.get(n) for n in f.needs)

    def _fusion_on(self, name: str, layer: str):
        """Record that the planner applied fusion `name` to `layer`."""
        self.fusions.setdefault(name, [])
        if layer not in self.fusions[name]:
            self.fusions[name].append(layer)

    # ------------------------------------------------------------------ shapes
    def sdims(self, level: int) -> Tuple[int, int, int]:
        s = self.img >> (level - 1)
        return (s, s, s) if self.dims == 3 else (1, s, s)

    def npix(self, level: int) -> int:
        d, h, w = self.sdims(level)
        return self.B * d * h * w

    def _buf(self, name, level, ch, dtype=None):
        dtype = self.adt if dtype is None else dtype
        d, h, w = self.sdims(level)
        shape = (self.B, h, w, ch) if self.dims == 2 else (self.B, d, h, w, ch)
        t = torch.empty(shape, dtype=dtype, device=self.device)
        self.bufs[name] = t
        return t

    # ------------------------------------------------------------------ weights
    def _alloc_weights(self):
        """bf16 arena with the conv kernels in their compute layouts + Adam pack segments."""
        spec, flat = self.spec, self.flat
        T = 3 ** self.dims
        Tt = 2 ** self.dims
        off = 0
        self.w_fwd_off: Dict[str, int] = {}
        self.w_dg_off: Dict[str, int] = {}
        layouts = {}
        for l in spec.param_layers():
            if l.kind == "conv":
                first = l.name == spec.layers[0].name
                ci_pad = self.cpad if first else l.cin
                row = _r64(T * ci_pad)                 # K padded to the 64-wide K step
                dgrow = _r64(T * l.cout)
                self.w_fwd_off[l.name] = off
                off += l.cout * row
                if not first:
                    self.w_dg_off[l.name] = off
                    off += l.cin * dgrow
                layouts[l.name] = (1, T, l.cin, l.cout, ci_pad, row, dgrow)
            elif l.kind == "tconv":
                row = _r64(l.cin)
                dgrow = _r64(Tt * l.cout)
                self.w_fwd_off[l.name] = off
                off += Tt * l.cout * row
                self.w_dg_off[l.name] = off
                off += l.cin * dgrow
                layouts[l.name] = (2, Tt, l.cin, l.cout, l.cin, row, dgrow)
        self.arena = torch.zeros(max(off, 64), dtype=self.adt, device=self.device)
        # the segments tile the whole flat buffer (Adam updates alignment gaps too):
        # a kind-0 segment absorbs the gap after it, a kernel segment gets its own
        segs = []
        ends = [e[2] for e in flat.entries[1:]] + [flat.numel]
        for (name, shape, foff, n), end in zip(flat.entries, ends):
            lname, var = name.split("/", 1)
            if var == "kernel" and lname in layouts:
                kind, t, ci, co, ci_pad, row, dgrow = layouts[lname]
                segs.append((foff, n, kind, t, ci, co, ci_pad, row, dgrow, 0,
                             self.w_fwd_off[lname], self.w_dg_off.get(lname, -1)))
                if end > foff + n:
                    segs.append((foff + n, end - foff - n, 0, 0, 0, 0, 0, 0, 0, 0, -1, -1))
            else:
                segs.append((foff, end - foff, 0, 0, 0, 0, 0, 0, 0, 0, -1, -1))
        dt = np.dtype([("off", "<i4"), ("n", "<i4"), ("kind", "<i4"), ("T", "<i4"), ("Ci", "<i4"),
                       ("Co", "<i4"), ("Ci_pad", "<i4"), ("rowstride", "<i4"), ("dg_rowstride", "<i4"),
                       ("pad_", "<i4"), ("fwd_off", "<i8"), ("dg_off", "<i8")])
        assert dt.itemsize == self.C.packseg_bytes()
        arr = np.array(segs, dtype=dt)
        self.seg_table = arr
        self.nseg = len(segs)
        self.segs = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)

    def wptr(self, lname, which="fwd"):
        off = self.w_fwd_off[lname] if which == "fwd" else self.w_dg_off[lname]
        return int(self.arena.data_ptr()) + 2 * off

    def master_ptr(self, varname):
        return int(self.flat.view(self.flat.master, varname).data_ptr())

    def grad_ptr(self, varname):
        return int(self.flat.view(self.flat.grad, varname).data_ptr())

    def repack(self, stream=None):
        """Refresh the bf16 compute copies from the fp32 master (no Adam)."""
        f = self.flat
        self.C.adam_pack(_ptr(f.master), _ptr(f.grad), _ptr(f.m), _ptr(f.v), f.numel,
                         _ptr(self.segs), self.nseg, 0.0, 0.9, 0.999, 1e-8, 1.0, 0,
                         _ptr(self.arena), native.stream_handle(stream), dtype=self.dt_id)

    def adam_step(self, lr, beta1_power, beta2_power, grad_scale=1.0, stream=None,
                  beta1=0.9, beta2=0.999, eps=1e-8):
        f = self.flat
        lr_t = lr * math.sqrt(1.0 - beta2_power) / (1.0 - beta1_power)
        if self.graphs is not None:
            # the captured launch reads {lr_t, gscale} from device memory
            self.adam_scalars[0].fill_(lr_t)
            self.adam_scalars[1].fill_(grad_scale)
            sc = _ptr(self.adam_scalars)
            self._replay(("adam", beta1, beta2, eps), lambda s: self.C.adam_pack(
                _ptr(f.master), _ptr(f.grad), _ptr(f.m), _ptr(f.v), f.numel, _ptr(self.segs), self.nseg,
                lr_t, beta1, beta2, eps, grad_scale, 1, _ptr(self.arena), s, sc, self.dt_id))
            return
        self.C.adam_pack(_ptr(f.master), _ptr(f.grad), _ptr(f.m), _ptr(f.v), f.numel,
                         _ptr(self.segs), self.nseg, lr_t, beta1, beta2, eps, grad_scale, 1,
                         _ptr(self.arena), native.stream_handle(stream), dtype=self.dt_id)

    # ------------------------------------------------------------------ buffers
    def _alloc_activations(self):
        spec = self.spec
        # channel-padded 16-bit input; load_batch casts the fp32 batch straight into it
        # (the pad channels stay zero)
        self._buf("x", 1, self.cpad).zero_()
        self.target = torch.zeros(self.npix(1), dtype=self.adt, device=self.device)
        # loss-gradient scale read by the head backward (fp16 dynamic loss scaling)
        self.loss_scale_dev = torch.ones(1, dtype=torch.float32, device=self.device)
        self._loss_scale = 1.0
        # tensor graph: name -> (level, channels, produced_by_relu, dropout)
        self.tinfo: Dict[str, Tuple[int, int, bool, bool]] = {"x": (1, self.cpad, False, False)}
        self.inputs: Dict[str, Tuple] = {}
        # upsampling decoder: the nearest upsample is materialised (elementwise ups_fwd) so
        # the decoder convs and their weight gradients run on the row-window kernels (the
        # round-1 address-generation fold measured slower and was removed)
        self.ups_materialize = True
        self.pool_codes: Dict[str, torch.Tensor] = {}
        cur = "x"
        pending_up = None
        for l in spec.layers:
            if l.kind == "conv":
                if l.skip_from is not None:
                    if pending_up is not None:
                        src1, up1 = pending_up, 2
                    else:
                        src1, up1 = cur, 1
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
                # first-argmax codes of the forward (one uint32 per pooled pixel x 8
                # channels): the backward reads these instead of the 4-8x larger input
                self.pool_codes[l.name] = torch.zeros(self.npix(l.level + 1) * l.cout // 8, dtype=torch.int32,
                                                      device=self.device)
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
        # ReLU bit masks (conv_params.h relu_bits): the forward of every ReLU conv whose
        # output masks a data gradient also writes 1 bit per element, and those data
        # gradients read the bits instead of the 16-bit activation -- at b1024 ~8 GB
        # less backward traffic.  Pool outputs need no mask at all: the pool backward
        # routes a gradient only where the window maximum is positive (code flag bits).
        self.relu_bits: Dict[str, torch.Tensor] = {}
        self.pool_outs = {l.name for l in spec.layers if l.kind == "pool"}
        # Head-on-load (head_grad.h): the head input's gradient dY = dlogit * w * (x > 0) is
        # rank-1 per pixel, so its consumers -- the data and weight gradients of the head's
        # input conv -- form it from the probability, target and the head input's ReLU bits
        # instead of reading a materialised 32-channel dY; the head backward only reduces
        # the Mask weight / bias gradients (on the side stream).  2D norm-free model with
        # a 32-channel head input on 16..128-wide rows (option head_onload=0: materialised).
        self.head_onload = self._fusion_ok("head_onload")
        if self.head_onload:
            self._fusion_on("head_onload", self.head_in)
        # head_wsum without head-on-load (3D): the head backward forms dY from the head
        # input's ReLU bits (head_dy), the input itself is not stored
        self._head_dy = not self.head_onload and not FUSIONS["head_wsum"].unmet(self)
        if spec.norm == "none":
            for l in spec.layers:
                if l.kind == "conv" and (l.name != self.head_in or self.head_onload or self._head_dy):
                    self.relu_bits[l.name] = torch.zeros(self.npix(l.level) * l.cout // 8, dtype=torch.uint8,
                                                         device=self.device)
        self._plan_tconv_fused()
        P = self.npix(1)
        self.prob = torch.zeros(P, dtype=torch.float32, device=self.device)
        nb = self.C.head_blocks(P)
        self.head_nb = nb
        hc = self.tinfo[self.head_in][1]
        self.head_partial = torch.zeros(nb * (hc + 1) + nb * 4, dtype=torch.float32, device=self.device)
        self.sums = torch.zeros(4, dtype=torch.float32, device=self.device)
        # gradient buffers: d:<tensor>, dskip:<tensor>, dfull:<tensor> (upsample fold)
        for name, (lvl, ch, _, _) in list(self.tinfo.items()):
            if name == "x" or name in self.tconv_fused:
                continue            # (a fused transposed conv's output gradient is never formed)
            if name == self.head_in and self.head_onload:
                continue            # (head-on-load: the head input's gradient is formed by its consumers)
            self.bufs["d:" + name] = torch.empty_like(self.bufs[name])
        # stand-in operand pointer of the head input's dgrad / wgrad under head-on-load
        # (never read: dY comes from prob / target / bits, the bias from the fused tile)
        self._no_dy = torch.zeros(64, dtype=self.adt, device=self.device)
        for l in spec.layers:
            if l.kind == "conv" and l.skip_from is not None:
                self.bufs["dskip:" + l.skip_from] = torch.empty_like(self.bufs[l.skip_from])
                src1, up1, _ = self.inputs[l.name]
                if up1 == 2:
                    lvl, ch = self.tinfo[src1][0], self.tinfo[src1][1]
                    d, h, w = self.sdims(l.level)
                    shape = (self.B, h, w, ch) if self.dims == 2 else (self.B, d, h, w, ch)
                    self.bufs["dfull:" + src1] = torch.empty(shape, dtype=self.adt, device=self.device)
                    if self.ups_materialize:
                        # nearest-upsampled copy read by the forward and the weight gradient
                        self.bufs["up:" + src1] = torch.empty(shape, dtype=self.adt, device=self.device)
        self.slab = None
        self.bias_slab = None
        self._alloc_norm()

    def _plan_tconv_fused(self):
        """Transposed convs whose backward runs composite (tconv_fused.hip): the data
        gradient of the tconv input is one coarse row-window conv over the space-to-depth
        image of the consumer conv's dz with weights composed from both layers (conv_win.h
        XF 4), the tconv weight / bias gradients come from 4x4-tap stride-2 slab sums
        through the chain rule -- the fine tconv output gradient (up to 1 GiB at b1024)
        is never written or re-read.  2D norm-free model; the consumer is the decoder conv
        whose skip-half data gradient rides on the pool backward.  Option tconv_fused = the
        deepest fine level fused (0 off)."""
        self.tconv_fused: Dict[str, dict] = {}
        self._dropped: Dict[str, torch.Tensor] = {}
        self._tf_consumer: Dict[str, str] = {}
        self._wa_chain_of: Dict[str, str] = {}  # consumer conv whose u-row wgrad is chained -> tconv
        self._ut_onload: Dict[str, str] = {}    # consumer conv that forms u on load -> tconv
        self._skip_onload: Dict[str, str] = {}  # skip source normalised on load (never stored) -> consumer
        self._ut_probe: Dict[str, dict] = {}
        top = self.opts["tconv_fused"]
        if not self._fusion_ok("tconv_fused") or (self.spec.norm != "none" and not self.fuse_norm_stats_planned()):
            return
        for l in self.spec.layers:
            if l.kind != "tconv" or l.level > top:
                continue
            cons = [x for x in self.spec.layers if x.kind == "conv" and self.inputs.get(x.name, ("",))[0] == l.name]
            if len(cons) != 1:
                continue
            c = cons[0]
            src1, up1, skip = self.inputs[c.name]
            has_pool = any(x.kind == "pool" and self.inputs[x.name][0] == skip for x in self.spec.layers)
            if up1 != 1 or skip is None or not has_pool or c.cout % 32 or l.cin % 32 or l.cout % 8:
                continue
            src = self.inputs[l.name][0]
            lo = self.sdims(l.level + 1)
            O, K = c.cout, l.cin
            rs = _r64(36 * O)
            probe = self._conv_common(l.level + 1, 3, 1, 1)
            probe.update(C1=4 * O, s2d=O, src1=1, wgt=1, Cout=K, relu=0, dst1=1, D1=K, mask1=1,
                         mask_bits=1 if src in self.relu_bits else 0)
            if self.spec.norm != "none":
                # normalised tconv input: the composite dgrad's epilogue is the dgrad-norm one
                probe.update(mask1=None, mask_bits=0, nz=1, na=1, nc=1, stats=1, npix=1,
                             ncs=0 if self.spec.norm == "batch" else K)
            try:
                if self.C.conv_fwd_grid(probe) <= 0:
                    continue
            except ValueError:
                continue
            self.tconv_fused[l.name] = dict(consumer=c.name, src=src, C=l.cout, K=K, O=O, Ca=c.cin, rs=rs,
                                            level=l.level,
                                            wg=torch.zeros(K * rs, dtype=self.adt, device=self.device),
                                            hs=torch.zeros(16 * O * K, dtype=torch.float32, device=self.device),
                                            bs=torch.zeros(16 * O, dtype=torch.float32, device=self.device))
            self._tf_consumer[c.name] = l.name
            self._fusion_on("tconv_fused", l.name)
            self._plan_wa_chain(l, c, self.tconv_fused[l.name])
            self._plan_ut_onload(l, c, self.tconv_fused[l.name])

    def fuse_norm_stats_planned(self):
        """Normalised model: every conv epilogue writes its statistics (the composite
        transposed-conv data gradient then carries the tconv input's norm backward rows)."""
        return getattr(self, "fuse_norm_stats", True)

    def _plan_wa_chain(self, l, c, tf):
        """Option tconv_wa (default 1): the weight gradient of the consumer conv
        z = conv3x3([u, skip]) of a composite-backward tconv u = tconv(b) takes its u rows
        from the 4x4-tap slab sums H / Bs the composite backward forms anyway (tconv_chain)
        and its skip rows from a skip-only weight gradient -- the u half of the wgrad (a
        1 GiB re-read at level 1) is gone (+3.0..3.2 %, r3_bench_history.md).  (The
        composite FORWARD on the coarse grid with composed weights measured -0.5..-1.2 %
        and was removed in round 4.)"""
        Cs, O = c.cin - l.cout, c.cout
        if not self._fusion_ok("tconv_wa", l.name) or Cs <= 0 or Cs % 32 or O % 16:
            return
        tf["wa"] = dict(Cs=Cs, skg=torch.zeros(9 * Cs * O, dtype=torch.float32, device=self.device))
        self._wa_chain_of[c.name] = l.name
        self._fusion_on("tconv_wa", l.name)

    def _ut_fields(self, tl, x_ptr):
        """conv_params.h TconvSrc fields: the consumer's src1 = tconv `tl` of x formed on load."""
        return dict(ut_x=x_ptr, ut_w=self.wptr(tl.name), ut_b=self.master_ptr(tl.name + "/bias"),
                    ut_C=tl.cin, ut_kpad=_r64(tl.cin))

    def _plan_ut_onload(self, l, c, tf):
        """Option tconv_onload (default 1): with the composite backward and the chained
        u-row weight gradient nothing but the consumer's forward reads u = tconv(b), so
        that forward forms each 32-channel chunk of u in LDS from b (conv_win.h XF 5): the
        transposed conv's forward launch and its fine output tensor (1 GiB at level 1,
        b1024) are gone, and the consumer reads the 4x smaller coarse b instead of u."""
        if l.level > self.opts["tconv_onload"] or not self._fusion_ok("tconv_onload", l.name):
            return
        normed = self.spec.norm != "none"
        d = self._conv_common(c.level, 3, 1, 1)
        d.update(C1=l.cout, C2=c.cin - l.cout, src1=1, src2=1, wgt=1, bias=1, Cout=c.cout,
                 relu=0 if normed else 1, dst1=1, **self._ut_fields(l, 1))
        if normed:
            d["stats"] = 1
        try:
            if self.C.conv_fwd_grid(d) <= 0:
                return
        except ValueError:
            return
        tf["ut"] = True
        self._ut_onload[c.name] = l.name
        self._fusion_on("tconv_onload", l.name)
        self._ut_probe[c.name] = d                # (skip_onload: decided once the norm buffers exist)
        # the fine output is never formed (no forward writes it, no backward reads it);
        # kept aside so the plan validation can flag any op that would still read it
        self._dropped[l.name] = self.bufs.pop(l.name, None)

    def _plan_skip_onload(self, c, d):
        """FUSIONS['skip_onload']: the normalised skip source S of the tconv-on-load consumer
        `c` (conv9a: BatchNorm, 128-wide rows) is never stored in training -- the consumer's
        persistent window normalises S's pre-norm z on load (conv_params.h x2a / x2b) and so
        does the chained skip-row weight gradient (the prefetching 128-wide window, xform 1);
        S's data gradient masks from z already (dgrad-norm epilogue), and norm_pool keeps only
        the pooled tensor.  Recorded in self._skip_onload {S: c}; the plan validation flags
        any op that would still read S's activation."""
        src1, up1, skip = self.inputs[c.name]
        if (skip is None or skip not in self.norm_layers or not self._fusion_ok("skip_onload", skip)
                or self.tinfo[skip][3] or self.tinfo[skip][1] != 32):
            return
        b = self.bufs
        xcs = 0 if self.spec.norm == "batch" else 32
        probe = dict(d, src2=1, x2a=_ptr(b["fa:" + skip]), x2b=_ptr(b["fc:" + skip]), x2cs=xcs)
        sd = self.sdims(c.level)
        wk = dict(N=self.B, QD=sd[0], QH=sd[1], QW=sd[2], AD=sd[0], AH=sd[1], AW=sd[2], KD=1, KH=3, KW=3,
                  stride=1, pad=1, upA=1, a1=_ptr(b["z:" + skip]), b=_ptr(b[skip]), M1=32, M2=0, Nc=c.cout,
                  splits=1, win=self.wgrad_win, bias_mode=1, pf=1, xform=1, xa=_ptr(b["fa:" + skip]),
                  xb=_ptr(b["fc:" + skip]), xcs=xcs)
        try:
            if self.C.conv_fwd_grid(probe) <= 0:
                return
            self.C.wgrad_validate(wk)
        except ValueError:
            return
        self._skip_onload[skip] = c.name
        self._fusion_on("skip_onload", skip)

    def _skip_xf_fields(self, skip, c, nb):
        """x2* fields of the tconv-on-load consumer reading skip source `skip` as pre-norm z."""
        b = self.bufs
        C = self.tinfo[skip][1]
        mo = 0 if self.spec.norm == "batch" else c * nb * C * 4       # per-sample [B][C] coefficients
        return dict(src2=_ptr(b["z:" + skip]) + self._toff(skip, c, nb), x2a=_ptr(b["fa:" + skip]) + mo,
                    x2b=_ptr(b["fc:" + skip]) + mo, x2cs=0 if self.spec.norm == "batch" else C)

    # ------------------------------------------------------------------ normalisation
    NORM_EPS = 1e-3          # models/reference.py::_norm (Keras default epsilon)
    BN_MOMENTUM = 0.01       # torch convention = Keras momentum 0.99

    def _alloc_norm(self):
        """Per normalised conv layer: the pre-norm conv output z:<L>, its gradient
        dz:<L>, per-(sample|batch, channel) mean / rstd saved for the backward,
        backward coefficients; BatchNorm running statistics (``self.state``, the
        same names as the ATen backend so checkpoints are interchangeable)."""
        self.state: Dict[str, torch.Tensor] = {}
        self.norm_layers = []
        # fused statistics (conv epilogues write per-tile partial sums): name -> buffer
        self._stat_bufs: Dict[str, torch.Tensor] = {}
        self._stat_retired: List[torch.Tensor] = []
        self._bwd_fused: Dict[str, Tuple[int, bool]] = {}
        self._dz_onload = set()              # norm layers whose dz the fused dgrad + wgrad forms on load
        self.fuse_norm_stats = True
        if self.spec.norm == "none":
            return
        f32 = torch.float32
        for l in self.spec.layers:
            if l.kind != "conv":
                continue
            self.norm_layers.append(l.name)
            self.bufs["z:" + l.name] = torch.empty_like(self.bufs[l.name])
            self.bufs["dz:" + l.name] = torch.empty_like(self.bufs[l.name])
            rows = 1 if self.spec.norm == "batch" else self.B
            # mean / rstd; relu-input coefficients fa / fc (u = fa z + fc, read by fused
            # consumers); backward coefficients ca / cb / cc
            for k in ("mean", "rstd", "fa", "fc", "ca", "cb", "cc"):
                self.bufs["%s:%s" % (k, l.name)] = torch.zeros(rows * l.cout, dtype=f32, device=self.device)
            if self.spec.norm == "batch":
                self.state[l.name + "/norm/moving_mean"] = torch.zeros(l.cout, dtype=f32, device=self.device)
                self.state[l.name + "/norm/moving_variance"] = torch.ones(l.cout, dtype=f32, device=self.device)

    def _stat_buf(self, key, floats):
        """Statistics buffer `key` of at least `floats` floats.  A buffer that has to grow is
        replaced, and the superseded one is kept alive (never freed under a recorded op) but
        is no named region: an op still pointing into it fails the plan's def-use check."""
        t = self._stat_bufs.get(key)
        if t is None or t.numel() < floats:
            if t is not None:
                self._stat_retired.append(t)
            t = torch.zeros(max(floats, 64), dtype=torch.float32, device=self.device)
            self._stat_bufs[key] = t
        return t

    def _fuse_stats(self, d, key, C, level, c=0, nb=None):
        """Let conv dict `d` write per-tile normalisation statistics from its epilogue
        (conv_epilogue.h EPI_STATS / EPI_DGRAD_NORM) if its kernel can.  Returns
        (rows, per_sample) or None; per_sample: every sample owns rows / N
        consecutive rows (required by GroupNorm's per-sample statistics).  Chunk c of
        nb images (the two-stream forward, d["N"] == nb) writes its rows after the rows
        of the chunks before it: sample-major, so the whole-batch row order is kept."""
        if not self.fuse_norm_stats:
            return None
        nb = nb or self.B
        try:
            rows, px = self.C.conv_stat_tiles(dict(d, stats=1))
        except ValueError:
            return None
        if rows == 0:
            return None
        P = self.npix(level) // self.B
        per_sample = px > 0 and P % px == 0 and rows % nb == 0
        if self.spec.norm == "group" and not per_sample:
            return None
        buf = self._stat_buf(key, (self.B // nb) * rows * 2 * C)
        d["stats"] = _ptr(buf) + c * rows * 2 * C * 4
        return rows, per_sample

    def _stat_rows(self, key, A, B, l, fused, plan, name, c=0, nb=None):
        """(rows pointer, row count) of the per-tile / per-block partial sums of layer l
        (images [c nb, (c + 1) nb)): the producer's epilogue rows when `fused`, else a
        moments pass over (A, A*B) -- A, B: pointers to the chunk's images."""
        nb = nb or self.B
        C, P = l.cout, self.npix(l.level) // self.B
        if fused:
            return _ptr(self._stat_bufs[key]) + c * fused[0] * 2 * C * 4, fused[0]
        R = nb * self.C.norm_blocks_per_sample(nb, P)
        rows = _ptr(self._stat_buf("m" + key, (self.B // nb) * R * 2 * C)) + c * R * 2 * C * 4
        plan.add_generic("norm_rows", [A, B, rows], [nb, P, C], [], name)
        return rows, R

    def _stat_work(self, key, R, C, c=0, nb=None):
        """Workspace of bn_stats / gn_stats (slices of R rows, or GroupNorm's per-sample
        parameter-gradient rows + their slices); one per forward chunk (the two chunks'
        finalizes run concurrently), each sized for the whole batch's rows so the
        one-stream evaluation plan never regrows (and frees) a buffer a recorded launch
        points into."""
        Rw = R * (self.B // (nb or self.B))
        # (+64: the single-launch finalize's hand-off counter past the slices, norm.hip)
        n = max(self.C.row_slices(Rw), 1) * 2 * C + self.B * 2 * C + self.C.row_slices(self.B) * 2 * C + 64
        return self._stat_buf("w" + key + (":%d" % c if c else ""), n)

    def _norm_fwd(self, plan, l, dropout, train, fused=None, c=0, nb=None):
        """z:<L> -> activation <L> = relu(norm(z)) (+ dropout) for images [c nb, (c+1) nb)
        (a chunk of the two-stream forward; GroupNorm only: per-sample statistics).
        fused: (rows, per_sample) when conv L's epilogue wrote the statistics (no
        separate moments pass)."""
        b, spec = self.bufs, self.spec
        nb = nb or self.B
        C, P, N = l.cout, self.npix(l.level) // self.B, nb
        z = b["z:" + l.name]
        zp = _ptr(z) + c * nb * P * C * z.element_size()
        mo = 0 if spec.norm == "batch" else c * nb * C * 4            # per-sample [B][C] coefficients
        mean, rstd = _ptr(b["mean:" + l.name]) + mo, _ptr(b["rstd:" + l.name]) + mo
        fa, fc = _ptr(b["fa:" + l.name]) + mo, _ptr(b["fc:" + l.name]) + mo
        gamma, beta = self.master_ptr(l.name + "/norm/gamma"), self.master_ptr(l.name + "/norm/beta")
        if spec.norm == "batch":
            assert nb == self.B, "BatchNorm statistics are whole-batch: no forward chunks"
            rm = self.state[l.name + "/norm/moving_mean"]
            rv = self.state[l.name + "/norm/moving_variance"]
            if train:
                rows, R = self._stat_rows("st:" + l.name, zp, zp, l, fused, plan, "bnstat:" + l.name)
            else:
                rows, R = _ptr(self._stat_buf("st:" + l.name, 64)), 1     # inference: running statistics
            ws = self._stat_work("st:" + l.name, R, C)
            plan.add_generic("bn_stats", [rows, gamma, beta, _ptr(rm), _ptr(rv), mean, rstd,
                                          fa, fc, 0, 0, 0, 0, 0, _ptr(ws)],
                             [R, C, 0 if train else 2], [float(N * P), self.NORM_EPS, self.BN_MOMENTUM],
                             "bnfin:" + l.name)
        else:
            rows, R = self._stat_rows("st:" + l.name, zp, zp, l, fused, plan, "gnstat:" + l.name, c, nb)
            ws = self._stat_work("st:" + l.name, R, C, c, nb)
            plan.add_generic("gn_stats", [rows, gamma, beta, mean, rstd, fa, fc, 0, 0, 0, 0, 0, _ptr(ws)],
                             [N, R // N, C, spec.groups, P, 0], [self.NORM_EPS], "gnfin:" + l.name)
        if l.name in self._xf_fwd:
            return          # the consumer conv normalises z on load and writes the activation
        if l.name == self.head_in and nb != self.B:
            # two-stream forward: the head (its loss sums need every pixel) runs on the
            # whole batch once both chunks are done (_build_forward_2s)
            self._deferred_head = (l, dropout, train)
            return
        self._norm_out(plan, l, dropout, train, c, nb)

    def _norm_out(self, plan, l, dropout, train, c=0, nb=None):
        """The pass after a layer's statistics: the normalised activation (with the 2x2
        max-pool of convNb; with the head logits / loss sums for the head input)."""
        b, spec = self.bufs, self.spec
        nb = nb or self.B
        C, P, N = l.cout, self.npix(l.level) // self.B, nb
        z = b["z:" + l.name]
        zp = _ptr(z) + c * nb * P * C * z.element_size()
        mo = 0 if spec.norm == "batch" else c * nb * C * 4
        mean, rstd = _ptr(b["mean:" + l.name]) + mo, _ptr(b["rstd:" + l.name]) + mo
        fa, fc = _ptr(b["fa:" + l.name]) + mo, _ptr(b["fc:" + l.name]) + mo
        gamma, beta = self.master_ptr(l.name + "/norm/gamma"), self.master_ptr(l.name + "/norm/beta")
        cstride = 0 if spec.norm == "batch" else C
        out = _ptr(b[l.name]) + self._toff(l.name, c, nb)
        if l.name == self.head_in and not (l.dropout and dropout) and self.tinfo[l.name][1] in (16, 32, 64):
            assert nb == self.B
            if train:
                # training: normalisation, logits, sigmoid, loss sums and the nine per-channel
                # pixel sums of the head's backward in one pass (head.hip norm_head_loss);
                # the activation is not stored -- nothing downstream reads it
                hp = self._stat_buf("hn:part", self.C.hn_partial_floats(N, P, C))
                plan.add_generic("norm_head_loss", [zp, fa, fc, self.master_ptr("Mask/kernel"),
                                                    self.master_ptr("Mask/bias"), _ptr(self.target), 0,
                                                    _ptr(self.prob), _ptr(hp), _ptr(self.sums)],
                                 [N, P, C, cstride], [], "fwd:Mask")
                self._norm_head_loss = True
                return
            # head input: normalisation + the 1x1 head's logits in one pass (head_finish follows)
            plan.add_generic("norm_head", [zp, fa, fc, self.master_ptr("Mask/kernel"),
                                           self.master_ptr("Mask/bias"), out, _ptr(self.prob)],
                             [self.npix(l.level), C, cstride, P], [], "norm:" + l.name)
            self._norm_head = True
            return
        pool = self._pool_of.get(l.name)
        if pool is not None and not (l.dropout and dropout):
            # convNb: normalisation and the 2x2 max-pool of its output in one pass
            dd, hh, ww = self.sdims(l.level)
            pcode = _ptr(self.pool_codes[pool]) + c * nb * (self.npix(l.level + 1) // self.B) * (C // 8) * 4
            if train and l.name in self._skip_onload:
                out = 0                      # (skip_onload: its consumers read z)
            plan.add_generic("norm_pool", [zp, fa, fc, out, _ptr(b[pool]) + self._toff(pool, c, nb), pcode],
                             [N, dd, hh, ww, C, int(self.dims == 3), cstride], [], "norm:" + l.name)
            self._pool_fused.add(pool)
            return
        plan.add_generic("norm_apply", [zp, mean, rstd, gamma, beta, out],
                         [N, P, C, cstride, 1, self._salt(l.name), 0, c * nb],
                         [spec.dropout if (l.dropout and dropout) else 0.0], "norm:" + l.name)

    def _norm_bwd_ops(self, l, apply=True):
        """Plan ops (callables) of d:<L> -> dz:<L> plus gamma/beta grads (apply=False:
        statistics and coefficients only -- conv L's data gradient forms dz on load)."""
        b, spec = self.bufs, self.spec
        C, P, N = l.cout, self.npix(l.level) // self.B, self.B
        g, z, dz = b["d:" + l.name], b["z:" + l.name], b["dz:" + l.name]
        mean, rstd = b["mean:" + l.name], b["rstd:" + l.name]
        ca, cb, cc = b["ca:" + l.name], b["cb:" + l.name], b["cc:" + l.name]
        gamma = self.master_ptr(l.name + "/norm/gamma")
        beta = self.master_ptr(l.name + "/norm/beta")
        dgam, dbet = self.grad_ptr(l.name + "/norm/gamma"), self.grad_ptr(l.name + "/norm/beta")
        fused = self._bwd_fused.get(l.name)
        ops = []

        hn = self._norm_head_loss and l.name == self.head_in

        def emit(pl):
            if hn:      # rows from the forward's head sums (head_norm_coef)
                rows, R = _ptr(self._hn_rows), N * self.C.hn_blocks_per_sample(N, P)
            else:
                rows, R = self._stat_rows("bst:" + l.name, _ptr(g), _ptr(z), l, fused, pl, "nstat_bwd:" + l.name)
            ws = self._stat_work("bst:" + l.name, R, C)
            if spec.norm == "batch":
                pl.add_generic("bn_stats", [rows, gamma, beta, 0, 0, _ptr(mean), _ptr(rstd), 0, 0,
                                            _ptr(ca), _ptr(cb), _ptr(cc), dgam, dbet, _ptr(ws)],
                               [R, C, 1], [float(N * P), self.NORM_EPS, self.BN_MOMENTUM], "bnfin_bwd:" + l.name)
                cstride = 0
            else:
                pl.add_generic("gn_stats", [rows, gamma, beta, _ptr(mean), _ptr(rstd), 0, 0, _ptr(ca),
                                            _ptr(cb), _ptr(cc), dgam, dbet, _ptr(ws)],
                               [N, R // N, C, spec.groups, P, 1], [self.NORM_EPS], "gnfin_bwd:" + l.name)
                cstride = C
            if not apply or l.name in self._dz_onload:
                return          # (dz formed on load by its consumers: conv_dw XF 2 / first-layer wgrad)
            if hn:      # dz = a w dlogit m + b z + c: g formed per pixel from prob and t
                fa, fc = b["fa:" + l.name], b["fc:" + l.name]
                pl.add_generic("head_norm_bwd", [_ptr(z), _ptr(self.prob), _ptr(self.target), _ptr(self.sums),
                                                 self.master_ptr("Mask/kernel"), _ptr(fa), _ptr(fc), _ptr(ca),
                                                 _ptr(cb), _ptr(cc), _ptr(dz), _ptr(self.loss_scale_dev)],
                               [N, P, C, cstride], [1.0 / float(N * P), self.bce_weight, 1.0],
                               "norm_bwd:" + l.name)
                return
            pl.add_generic("norm_bwd_apply", [_ptr(g), _ptr(z), _ptr(ca), _ptr(cb), _ptr(cc), _ptr(dz)],
                           [N, P, C, cstride], [], "norm_bwd:" + l.name)
        ops.append(emit)
        return ops

    def _head_grad_fields(self):
        """hg_* fields (conv_params.h HeadGrad) of the head input's gradient consumers."""
        return dict(hg_prob=_ptr(self.prob), hg_t=_ptr(self.target), hg_sums=_ptr(self.sums),
                    hg_w=self.master_ptr("Mask/kernel"),
                    hg_bits=_ptr(self.relu_bits[self.head_in]) if self.head_in in self.relu_bits else None,
                    hg_gscale=_ptr(self.loss_scale_dev), hg_inv_total=1.0 / float(self.npix(1)),
                    hg_bce_w=self.bce_weight)

    def _tail_halves(self, d, l, src1, skip, dy):
        """Two half-batch copies of dgrad dict `d` when its destination is the first
        layer's output (the last dgrad of the backward) and the halves line up with
        the first layer's weight-gradient splits (norm-free 2D model, even batch), else
        None."""
        if skip is not None or self.inputs.get(src1, ("",))[0] != "x" or not self._fusion_ok("tail_halves"):
            return None      # (the first-layer row-window wgrad, whose split halves are image halves)
        b = self.bufs

        def half(t):
            return t.numel() * t.element_size() // 2

        mk = self.relu_bits.get(src1, b[src1]) if d.get("mask1") else None
        h1 = dict(d, N=self.B // 2)
        h2 = dict(h1, src1=d["src1"] + half(dy), dst1=d["dst1"] + half(b["d:" + src1]))
        if mk is not None:
            h2["mask1"] = d["mask1"] + half(mk)
        try:
            for h in (h1, h2):
                self.C.conv_fwd_grid(h)
        except ValueError:
            return None
        self._fusion_on("tail_halves", l.name)
        return h1, h2

    def _plan_dw_fuse(self, l, src1, skip, parts, wspec):
        """Fused data + weight gradient (conv_dw.hip, FUSIONS['dw_fused']): the data
        gradient dict(s) `parts` of conv `l` (one, or the two batch halves of the tail split)
        also produce the weight-gradient partials of `wspec` from the dY halo they stage --
        dY (1 GiB at level 1, b1024) is read once instead of twice.  Returns the dicts with
        the fw_* fields (slab pointers filled at emission), or None."""
        if (not self._fusion_ok("dw_fused") or skip is not None or l.cin != 32 or l.cout != 32
                or wspec.get("kernel_out") or wspec["kd"].get("xform")
                or wspec["M1"] != 32 or wspec["M2"] or src1 not in self.bufs):
            return None
        nsplit = self.opts["dw_wgs"]
        b = self.bufs
        half = b[src1].numel() * b[src1].element_size() // len(parts)
        if len(parts) > 1 and parts[0].get("nz"):
            return None          # (the statistics rows of the dgrad-norm epilogue are per whole launch)
        out = []
        for k, d in enumerate(parts):
            if d.get("route_gy") or (d.get("hg_prob") and len(parts) > 1):
                return None       # (head-on-load: the head input's dY formed from prob / target / bits, XF 4)
            f = dict(d, rev=0, fw_x=_ptr(b[src1]) + k * half, fw_Cx=l.cin, fw_nsplit=nsplit, fw_split_lo=k * nsplit,
                     name=d["name"])
            if f.get("nz") and not self._restat_dgrad_norm(f, src1):
                return None
            try:
                if self.C.conv_fwd_grid(dict(f, fw_slab=1, fw_bias_slab=1)) != nsplit:
                    return None
            except ValueError:
                return None
            out.append(f)
        wspec["dw"] = dict(rows=nsplit * len(parts))
        self._fusion_on("dw_fused", l.name)
        if len(out) == 1 and l.name in self.norm_layers and self._fusion_ok("dz_onload", l.name):
            # the conv's own norm backward on load: the halo is formed from g and z (XF 2), or
            # for the normalised head input from z, the probability and the target (XF 3: g
            # is never formed either -- head_norm_bwd's pass disappears)
            C = l.cout
            xf = dict(out[0], xform=2, src1=_ptr(b["d:" + l.name]), xz=_ptr(b["z:" + l.name]),
                      xa=_ptr(b["ca:" + l.name]), xb=_ptr(b["cb:" + l.name]), xc=_ptr(b["cc:" + l.name]),
                      xcs=0 if self.spec.norm == "batch" else C)
            if self._norm_head_loss and l.name == self.head_in:
                hg = self._head_grad_fields()
                hg.pop("hg_bits")
                xf.update(hg, src1=_ptr(b["z:" + l.name]), hg_fa=_ptr(b["fa:" + l.name]),
                          hg_fc=_ptr(b["fc:" + l.name]))
            try:
                ok = self.C.conv_fwd_grid(dict(xf, fw_slab=1, fw_bias_slab=1)) == nsplit
            except ValueError:
                ok = False
            if ok:
                out = [xf]
                self._dz_onload.add(l.name)
                self._fusion_on("dz_onload", l.name)
        return out

    def _dz_split_fields(self, l, src1, skip):
        """xform-2 fields (dz = ca g + cb z + cc formed on load from g = d:<l>) when conv `l`'s
        dz is read by nothing but its own data gradient and weight gradient and both kernels
        take the transform (FUSIONS['dz_split']): single-source 2D conv on 16..64-wide rows,
        no fused data + weight gradient, no chained / composite consumer; else None.  The
        decision is recorded (_dz_onload): no norm_bwd_apply pass, dz is never stored."""
        if (not self._fusion_ok("dz_split") or skip is not None or l.name not in self.norm_layers
                or self.inputs.get(l.name, ("",))[1] != 1 or l.name in self._wa_chain_of
                or l.name in self._tf_consumer or (self._norm_head_loss and l.name == self.head_in)):
            return None
        W = self.sdims(l.level)[2]
        if W < 16 or W > 64 or l.cin % 32 or l.cout % 32:
            return None
        b = self.bufs
        xf = dict(xform=2, xa=_ptr(b["ca:" + l.name]), xb=_ptr(b["cb:" + l.name]), xc=_ptr(b["cc:" + l.name]),
                  xz=_ptr(b["z:" + l.name]), xcs=0 if self.spec.norm == "batch" else l.cout)
        # kernel probes: the data gradient (with its dgrad-norm epilogue, as planned) and the
        # weight gradient, both with the transform
        d = self._conv_common(l.level, 3, 1, 1)
        lvl, ch, relu_src, drop = self.tinfo[src1]
        m1, mb = self._relu_mask(src1) if relu_src else (None, 0)
        d.update(name="dgrad:" + l.name, C1=l.cout, src1=_ptr(b["d:" + l.name]), wgt=self.wptr(l.name, "dg"),
                 Cout=l.cin, relu=0, dst1=_ptr(b["d:" + src1]), D1=l.cin, mask1=m1, mask_bits=mb)
        d.update(xf)                  # (the planned dgrad may carry the dgrad-norm epilogue: both take XF 2)
        sd = self.sdims(l.level)
        kd = dict(N=self.B, QD=sd[0], QH=sd[1], QW=sd[2], AD=sd[0], AH=sd[1], AW=sd[2], KD=1, KH=3, KW=3,
                  stride=1, pad=1, upA=1, a1=_ptr(b[src1]), b=_ptr(b["d:" + l.name]), M1=l.cin, M2=0, Nc=l.cout,
                  splits=1, win=self.wgrad_win, bias_mode=1, **xf)
        try:
            self.C.conv_fwd_grid(d)
            self.C.wgrad_validate(kd)
        except ValueError:
            return None
        self._dz_onload.add(l.name)
        self._fusion_on("dz_split", l.name)
        return xf

    def _restat_dgrad_norm(self, f, tname):
        """Fused data + weight gradient `f` whose epilogue is the dgrad-norm one (gradient of
        normalised activation `tname`): its statistics rows are per 256-pixel window, not
        the split kernel's tiles -- re-plan them (rows + buffer) for the fused launch."""
        l = next(x for x in self.spec.layers if x.name == tname)
        d = dict(f, fw_slab=1, fw_bias_slab=1)       # (slab pointers: filled at emission)
        d.pop("stats", None)
        fused = self._fuse_stats(d, "bst:" + tname, l.cout, l.level)
        if fused is None:
            return False
        f["stats"] = d["stats"]
        self._bwd_fused[tname] = fused
        return True

    def _skip_route(self, l, skip, c1, c2, dy):
        """(pool name, dgrad dict) of the deferred skip half of decoder conv l's data
        gradient when it can carry the pool backward of its skip source (row-window
        data gradient; 3D with option route3), else None (the dual-destination dgrad + separate pool backward).  Saves the skip-gradient tensor's
        write and re-read: the pool backward's read of it becomes a second read of dy."""
        if not self._fusion_ok("skip_route"):
            return None
        if self.spec.norm != "none" and not (skip in self.norm_layers and self.fuse_norm_stats):
            return None
        pool = next((x.name for x in self.spec.layers if x.kind == "pool" and self.inputs[x.name][0] == skip), None)
        if pool is None:
            return None
        b = self.bufs
        m, mb = self._relu_mask(skip)
        dgrow = _r64((3 ** self.dims) * l.cout)
        d = self._conv_common(l.level, 3, 1, 1)
        d.update(name="dgrad_skip:" + l.name, C1=l.cout, src1=_ptr(dy),
                 wgt=self.wptr(l.name, "dg") + 2 * c1 * dgrow, Cout=c2, relu=0,
                 dst1=_ptr(b["d:" + skip]), D1=c2, mask1=m, mask_bits=mb, route_gy=_ptr(b["d:" + pool]),
                 pool_code=_ptr(self.pool_codes[pool]))
        if self.spec.norm != "none":
            # normalised skip source: the epilogue also recomputes the ReLU mask from the
            # pre-norm z and writes the norm backward's {sum g, sum g z} rows (the
            # pool_bwd_norm pass and the skip-gradient tensor are gone)
            saved = dict(self._bwd_fused)
            self._fuse_dgrad_norm(d, skip)
            if not d.get("nz"):
                self._bwd_fused = saved
                return None
        try:
            self.C.conv_fwd_grid(d)
        except ValueError:
            self._bwd_fused.pop(skip, None)
            return None
        if self.spec.norm == "none":
            self._rev_order(d, "g:" + l.name, "g:" + skip)
        self._fusion_on("skip_route", l.name)
        return pool, d

    def _relu_mask(self, tname):
        """(mask pointer, is-bits) of the ReLU mask a data gradient into tensor `tname`
        applies: its bit tensor when the forward writes one, none for a pool output
        (norm-free model: the pool backward routes only to positive maxima), else the
        16-bit activation itself."""
        if tname in self.relu_bits:
            return _ptr(self.relu_bits[tname]), 1
        if tname in self.pool_outs and self.spec.norm == "none":
            return None, 0
        return _ptr(self.bufs[tname]), 0

    def _fuse_dgrad_norm(self, d, tname):
        """dgrad dict `d` writes the gradient of tensor `tname`: when that is a
        normalised conv output, let its epilogue recompute the ReLU / dropout mask
        from the pre-norm z and emit the backward statistics (no nstat_bwd pass)."""
        if tname not in self.norm_layers:
            return
        l = next(x for x in self.spec.layers if x.name == tname)
        C = l.cout
        d2 = dict(d, mask1=None, mask_bits=0, mask_scale1=1.0, nz=_ptr(self.bufs["z:" + tname]),
                  na=_ptr(self.bufs["fa:" + tname]), nc=_ptr(self.bufs["fc:" + tname]),
                  ncs=0 if self.spec.norm == "batch" else C, npix=self.npix(l.level) // self.B,
                  nd_rate=self.spec.dropout if self.tinfo[tname][3] else 0.0, nd_salt=self._salt(tname))
        fused = self._fuse_stats(d2, "bst:" + tname, C, l.level)
        if fused is None:
            return
        d.clear()
        d.update(d2)
        self._bwd_fused[tname] = fused

    # ------------------------------------------------------------------ plans
    def _conv_common(self, level, K, stride, pad, out_level=None, in_level=None):
        od, oh, ow = self.sdims(out_level or level)
        idd, ih, iw = self.sdims(in_level or level)
        kd = K if self.dims == 3 else 1
        return dict(N=self.B, OD=od, OH=oh, OW=ow, ID=idd, IH=ih, IW=iw, KD=kd, KH=K, KW=K,
                    stride=stride, pad=pad, tile=0, win_pf=self.opts["win_pf"],
                    win_cp=self.opts["win_cp3"] if self.dims == 3 else self.opts["win_cp"])

    def _salt(self, lname):
        return [l.name for l in self.spec.layers].index(lname)

    def _toff(self, tname, c, nb):
        """Byte offset of image c*nb of activation tensor `tname`."""
        lvl, ch = self.tinfo[tname][0], self.tinfo[tname][1]
        d, h, w = self.sdims(lvl)
        return c * nb * d * h * w * ch * self.bufs[tname].element_size()

    def _xf_fwd_fields(self, src, c=0, nb=None, dropout=False):
        """Operand-transform fields of a conv reading normalised activation `src` as the
        pre-norm z (conv_params.h xform 1) for images [c nb, (c + 1) nb); the conv also
        writes the activation (with `src`'s dropout when `dropout`: xd_*, norm_apply's keep
        mask of the whole-batch element index)."""
        b = self.bufs
        nb = nb or self.B
        C = self.tinfo[src][1]
        mo = 0 if self.spec.norm == "batch" else c * nb * C * 4       # per-sample [B][C] coefficients
        out = dict(xform=1, xa=_ptr(b["fa:" + src]) + mo, xb=_ptr(b["fc:" + src]) + mo,
                   xcs=0 if self.spec.norm == "batch" else C,
                   xout=_ptr(b[src]) + self._toff(src, c, nb))
        if dropout and self.tinfo[src][3] and self.spec.dropout > 0:
            P = self.npix(self.tinfo[src][0]) // self.B
            out.update(xd_rate=self.spec.dropout, xd_salt=self._salt(src), xd_idx0=c * nb * P * C)
        return out

    def _plan_xforms(self):
        """Normalised activations whose only consumer is the next conv's first source
        (the 'a' convs of each block; with dropout only under option xf_drop): that conv normalises z on load and
        also stores the activation for its weight gradient (+0.4 % BN b1024 over a
        separate norm_apply pass).  Decided once, for the training and the evaluation
        plans alike.  (Measured and dropped in round 2: the consumer's weight gradient
        normalising on load too, -1.3 % BN / -1.5 % GN; dz formed on load by the data
        gradient, -1.1 % BN; level-1 dgrad + wgrad both forming dz, -1.2 % BN.  Round 6 rebuilt
        the last two: level 1 in the fused conv_dw window (kept), levels 2-4 in the split
        consumers -- option dz_split, -3.2 % BN, off.)"""
        self._xf_fwd = set()
        if not self._fusion_ok("norm_onload"):
            return
        users: Dict[str, list] = {}
        for name, inp in self.inputs.items():
            for k, t in enumerate(inp[:1] + inp[2:3]):
                if t:
                    users.setdefault(t, []).append((name, k))
        users.setdefault(self.head_in, []).append(("Mask", 0))
        kinds = {l.name: l.kind for l in self.spec.layers}
        for l in self.spec.layers:
            if l.kind != "conv" or l.name not in self.norm_layers or (self.tinfo[l.name][3] and not
                                                                      self.opts["xf_drop"]):
                continue
            u = users.get(l.name, [])
            if len(u) != 1 or u[0][1] != 0 or kinds.get(u[0][0]) != "conv":
                continue
            l2 = next(x for x in self.spec.layers if x.name == u[0][0])
            src1, up1, skip = self.inputs[l2.name]
            if skip or up1 != 1:
                continue
            d = self._conv_common(l2.level, 3, 1, 1)
            d.update(C1=l.cout, src1=_ptr(self.bufs["z:" + l.name]), wgt=self.wptr(l2.name), Cout=l2.cout,
                     relu=0, dst1=_ptr(self.bufs["z:" + l2.name]), bias=self.master_ptr(l2.name + "/bias"))
            d.update(self._xf_fwd_fields(l.name, dropout=True))
            try:
                self.C.conv_fwd_grid(d)
            except ValueError:
                continue
            self._xf_fwd.add(l.name)
            self._fusion_on("norm_onload", l.name)

    # (option fwd_offset: the second forward chunk starts after the first chunk's first
    # fwd_offset layers; round-2 sweep 3 / 6 / 9 / 13: -0.2 / +0.3 / . / -0.6 %)

    def _fwd_streams(self, train):
        """2: the training forward runs as two half-batch chunks on two HIP streams, the
        second chunk started once the first has finished its first fwd_offset layers, so
        kernels of different levels (bandwidth-bound full-resolution ones, MFMA-bound
        coarse ones) share the GPU.  Norm-free or GroupNorm model (per-sample statistics:
        each chunk finalizes its own samples; the head's loss sums run on the whole batch
        after both chunks) with an even batch -- BatchNorm needs whole-batch statistics;
        option fwd_streams=1 keeps one stream.  Default 2 since round 3: same-box
        interleaved A/B of the headline step +1.0 / +1.0 / +0.6 % (44.2k -> 44.7k img/s,
        round 2 measured +0.9 % the same way).  (A CPU dry run plans it too, for the
        static plan validation.)"""
        if not train or not self._fusion_ok("fwd_2streams") or (self.device.type != "cuda" and not self._dry):
            return 1
        return 2

    def _build_forward(self, plan, dropout, train=True):
        spec = self.spec
        nst = self._fwd_streams(train) if plan is self.plan else 1
        if nst == 2:
            return self._build_forward_2s(plan, dropout, train)
        # fused head: the Mask 1x1 conv + sigmoid + loss partials run in the epilogue of
        # the head's input conv (option head_fuse=0 keeps the separate head launch)
        self._head_fused_blocks = 0
        self._norm_head = False
        if train:
            self._norm_head_loss = False
        self._fuse_head = self._fusion_ok("head_fuse")
        # convNb -> 2x2 max-pool fused into the conv's epilogue where the kernel can
        self._pool_of = {self.inputs[x.name][0]: x.name for x in spec.layers if x.kind == "pool"}
        self._pool_fused = set()
        for l in spec.layers:
            if l.kind != "up":
                self._fwd_layer(plan, l, dropout, train, 0, self.B)

    def _build_forward_2s(self, plan, dropout, train):
        """Plan order: chunk 0's layers, chunk 1's layers, then the head finish on the
        whole batch (its loss partials need every pixel); forward() launches the two
        chunks on two streams."""
        spec = self.spec
        self._head_fused_blocks = 0
        self._norm_head = False
        self._fuse_head = self._fusion_ok("head_fuse")
        self._pool_of = {self.inputs[x.name][0]: x.name for x in spec.layers if x.kind == "pool"}
        self._pool_fused = set()
        layers = [l for l in spec.layers if l.kind not in ("up", "mask")]
        nb = self.B // 2
        off = self.opts["fwd_offset"]
        self._fwd2 = []                      # (first op, op after the offset layers, end) per chunk
        self._deferred_head = None
        for c in range(2):
            start = plan.size()
            mark = start
            for k, l in enumerate(layers):
                self._fwd_layer(plan, l, dropout, train, c, nb)
                if k + 1 == off:
                    mark = plan.size()
            self._fwd2.append((start, mark, plan.size()))
        if self._deferred_head is not None:
            # GroupNorm: the head input's normalisation with the head logits / loss sums on
            # the whole batch (both chunks' per-sample statistics are in place by now)
            self._norm_out(plan, *self._deferred_head)
            self._deferred_head = None
        for l in spec.layers:
            if l.kind == "mask":
                self._fwd_layer(plan, l, dropout, train, 0, self.B)

    def _fwd_layer(self, plan, l, dropout, train, c, nb):
        """Forward launches of layer `l` for images [c*nb, (c+1)*nb)."""
        spec = self.spec
        b = self.bufs
        nch = self.B // nb

        def P(t):
            return None if t is None else _ptr(b[t]) + self._toff(t, c, nb)

        if l.kind == "conv":
            src1, up1, skip = self.inputs[l.name]
            c1 = self.tinfo[src1][1]
            s1 = None if l.name in self._ut_onload else P(src1)
            if up1 == 2 and self.ups_materialize:
                lvl = self.tinfo[src1][0]
                dd, hh, ww = self.sdims(lvl)
                fd, fh, fw = self.sdims(l.level)
                s1 = _ptr(b["up:" + src1]) + c * nb * fd * fh * fw * c1 * b["up:" + src1].element_size()
                plan.add_generic("ups_fwd", [P(src1), s1], [nb, dd, hh, ww, c1, int(self.dims == 3)], [],
                                 "fwd:up:" + src1)
                up1 = 1
            d = self._conv_common(l.level, 3, 1, 1)
            d["N"] = nb
            normed = spec.norm != "none"
            ut = self._ut_onload.get(l.name)
            if ut is not None:
                tl = next(x for x in spec.layers if x.name == ut)
                d.update(self._ut_fields(tl, P(self.inputs[ut][0])))
                s1 = d["ut_x"]
            skip_xf = train and skip is not None and self._skip_onload.get(skip) == l.name
            if src1 in self._xf_fwd:
                d.update(self._xf_fwd_fields(src1, c, nb, dropout))
                s1 = _ptr(b["z:" + src1]) + self._toff(src1, c, nb)
            d.update(name="fwd:" + l.name, C1=c1, C2=self.tinfo[skip][1] if skip else 0, up1=up1,
                     src1=s1, src2=P(skip) if skip else None,
                     wgt=self.wptr(l.name), bias=self.master_ptr(l.name + "/bias"),
                     Cout=l.cout, relu=0 if normed else 1,
                     dst1=_ptr(b["z:" + l.name]) + self._toff(l.name, c, nb) if normed else P(l.name),
                     drop_rate=spec.dropout if (l.dropout and dropout and not normed) else 0.0,
                     salt=self._salt(l.name), drop_idx0=c * nb * (self.npix(l.level) // self.B) * l.cout)
            if skip_xf:
                d.update(self._skip_xf_fields(skip, c, nb))
            bits = self.relu_bits.get(l.name)
            if bits is not None and not normed:
                d["relu_bits"] = _ptr(bits) + c * nb * (self.npix(l.level) // self.B) * l.cout // 8
            pool = self._pool_of.get(l.name)
            if pool is not None and self._fusion_ok("pool_epilogue") and (nch == 1 or self._fwd2_active(plan)):
                # fused 2x2 max-pool: the epilogue writes the pooled tensor + argmax codes
                pcode = _ptr(self.pool_codes[pool]) + c * nb * (self.npix(l.level + 1) // self.B) * (l.cout // 8) * 4
                dp = dict(d, pool_dst=P(pool), pool_code=pcode)
                try:
                    self.C.conv_fwd_grid(dp)
                    d = dp
                    self._pool_fused.add(pool)
                    self._fusion_on("pool_epilogue", l.name)
                except ValueError:
                    pass
            if l.name == self.head_in and self._fuse_head and not d["drop_rate"]:
                nbk = self._head_grid(d)
                if nbk:
                    self._fusion_on("head_fuse", l.name)
                    d.update(head_w=self.master_ptr("Mask/kernel"), head_b=self.master_ptr("Mask/bias"),
                             head_logit=_ptr(self.prob) + 4 * c * nb * (self.npix(1) // self.B))
                    self._head_fused_blocks = nbk
                    if train:
                        self._plan_head_wsum(d, l, c, nb, nch)
            self._rev_order(d, src1, l.name, pool if pool in self._pool_fused else None)
            fused = None
            if normed and (train or spec.norm == "group"):
                fused = self._fuse_stats(d, "st:" + l.name, l.cout, l.level, c, nb)
            plan.add_conv_fwd(d)
            if normed:
                self._norm_fwd(plan, l, dropout, train, fused, c, nb)
        elif l.kind == "pool" and l.name in self._pool_fused:
            pass                                 # written by its source conv's epilogue
        elif l.kind == "pool":
            src = self.inputs[l.name][0]
            dd, hh, ww = self.sdims(l.level)
            pd, ph, pw = self.sdims(l.level + 1)
            code = _ptr(self.pool_codes[l.name]) + c * nb * pd * ph * pw * (l.cout // 8) * 4
            plan.add_generic("pool_fwd", [P(src), P(l.name), code],
                             [nb, dd, hh, ww, l.cout, int(self.dims == 3)], [], "fwd:" + l.name)
        elif l.kind == "tconv" and l.name in self._ut_onload.values():
            pass                                 # formed on load by its consumer's forward
        elif l.kind == "tconv":
            src = self.inputs[l.name][0]
            d = self._conv_common(l.level + 1, 1, 1, 0)
            d["N"] = nb
            d.update(name="fwd:" + l.name, C1=l.cin, src1=P(src), wgt=self.wptr(l.name),
                     bias=self.master_ptr(l.name + "/bias"), Cout=(2 ** self.dims) * l.cout,
                     relu=0, shuffle=self.dims, dst1=P(l.name))
            plan.add_conv_fwd(d)
        elif l.kind == "mask" and train and self._norm_head_loss:
            pass                                 # loss sums written by norm_head_loss
        elif l.kind == "mask" and (self._head_fused_blocks or self._norm_head):
            plan.add_generic("head_finish", [_ptr(self.prob), _ptr(self.target), _ptr(self.head_partial),
                                             _ptr(self.sums)], [self.npix(1)], [], "fwd:Mask")
        elif l.kind == "mask":
            P1 = self.npix(1)
            hc = self.tinfo[self.head_in][1]
            part = self.head_partial
            plan.add_generic("head_fwd", [_ptr(b[self.head_in]), self.master_ptr("Mask/kernel"),
                                          self.master_ptr("Mask/bias"), _ptr(self.target),
                                          _ptr(self.prob), _ptr(part), _ptr(self.sums)],
                             [P1, hc], [], "fwd:Mask")

    def _rev_order(self, d, src, out, *also):
        """_rev_mode bit 0 (forward) / bit 1 (data gradients): a row-window conv
        walks its windows in the reverse of the order its input was written in, so it
        starts on the producer's most recent output -- still in the Infinity Cache at
        sizes far beyond it.  Records the order `out` (and `also`) were written in.
        Default 3 (both): same-box sweep of the headline step +0.5 % (bit 0 or 1
        alone +0.3 %); the windows' results are bit-identical either way."""
        if not hasattr(self, "_rev_of"):
            self._rev_of = {}
        bit = 2 if d.get("name", "").startswith("dgrad") else 1
        r = 0
        if self._rev_mode & bit:
            r = 1 - self._rev_of.get(src, 0)
            try:
                if self.C.conv_fwd_grid(dict(d, rev=r)) > 0:
                    d["rev"] = r
                else:
                    r = 0
            except ValueError:
                r = 0
        for t in (out,) + also:
            if t is not None:
                self._rev_of[t] = r

    def _fwd2_active(self, plan):
        return plan is self.plan and getattr(self, "_fwd2", None) is not None and self._fwd_streams(True) == 2

    def _plan_head_wsum(self, d, l, c, nb, nch):
        """FUSIONS['head_wsum']: the fused-head forward of chunk c also accumulates the Mask
        weight-gradient sums (one 100-float row per workgroup into self.head_ws) and does not
        store the head input -- its only other reader was the head backward's weight
        gradient (head-on-load: the data gradients form dY from the probability, target and
        ReLU bits).  `d` is updated in place when the kernel takes it."""
        if not self._fusion_ok("head_wsum", l.name):
            return
        P = self.npix(1) // self.B
        probe = dict(d, head_t=_ptr(self.target), head_ws=1, head_nostore=1, dst1=None)
        try:
            grid = int(self.C.conv_fwd_grid(probe))
        except ValueError:
            return
        if grid <= 0:
            return
        if getattr(self, "head_ws", None) is None or self.head_ws.numel() < nch * grid * 100:
            self.head_ws = torch.zeros(nch * grid * 100, dtype=torch.float32, device=self.device)
            self._head_ws_rows = 0
        d.update(head_t=_ptr(self.target) + 2 * c * nb * P, head_ws=_ptr(self.head_ws) + 4 * c * grid * 100,
                 head_ws_rows=grid, head_nostore=1, dst1=None)
        self._head_ws_rows = max(self._head_ws_rows, (c + 1) * grid)
        self._fusion_on("head_wsum", l.name)

    def _head_grid(self, d):
        """Workgroups of the head-input conv when its forward can carry the fused
        head (32-channel ReLU row-window launch), else 0."""
        if self.tinfo[self.head_in][1] != 32:
            return 0
        try:
            return int(self.C.conv_fwd_grid(dict(d, head_w=1, head_b=1, head_logit=1)))
        except ValueError:
            return 0

    @staticmethod
    def _colsum_blocks(rows, C):
        return max(1, min(512, rows // 256))

    def _wgrad_pick(self, w):
        """Tile config of a wgrad spec; QW marks 2D 3x3 convs (row-window candidates)."""
        return self.C.wgrad_pick(w["M1"], w["M2"], w["Nc"], w["KT"], QW=w.get("QW", 0), upA=w.get("upA", 1),
                                 win=self.wgrad_win, QH=w.get("QH", 0), QD=w.get("QD", 0),
                                 xform=w["kd"].get("xform", 0) if "kd" in w else 0)

    def _wgrad_splits(self, w):
        M1, M2, Nc, KT, Q = w["M1"], w["M2"], w["Nc"], w["KT"], w["Q"]
        BM, BN, NTAP, smallc = self._wgrad_pick(w)
        Mtot = ((KT * M1 + BM - 1) // BM) * BM if smallc else M1 + M2
        tg = 1 if smallc else KT // NTAP
        tiles = (Mtot // BM) * (Nc // BN) * tg
        # ~2 workgroups per CU: enough to fill 256 CUs, few enough that the fp32
        # split-K slabs stay small next to the GEMM's own operand traffic
        splits = max(1, min(-(-self.wg_target // tiles), max(1, Q // (64 * 16))))
        taps = 1 if smallc else KT
        return splits, Mtot, taps, tg, smallc

    def _build_backward(self, plan):
        """Backward ops are first collected as closures (slab sizes are only known
        after every wgrad is sized), then emitted in order."""
        ops = []  # list of callables(plan) in emission order, plus layer-complete markers
        spec = self.spec
        b = self.bufs
        P1 = self.npix(1)
        layers = spec.layers
        KT3 = 3 ** self.dims
        KT2 = 2 ** self.dims
        inv_total = 1.0 / float(P1)

        def emit_generic(kind, ptrs, ints, floats, name):
            ops.append(lambda pl: pl.add_generic(kind, ptrs(), ints, floats, name))

        def emit_conv(d):
            ops.append(lambda pl: pl.add_conv_fwd(d()))

        wg_specs = []

        def emit_wgrad(args):
            wg_specs.append(args)
            idx = len(wg_specs) - 1
            ops.append(("wgrad", idx))

        def done(lname):
            ops.append(("done", lname))

        def src_normed(t):
            return t in self.norm_layers and self.fuse_norm_stats

        self._deferred_skip = {}
        tail_parts = {}
        for tname, tf in self.tconv_fused.items():
            # composite data-gradient weights from this step's fp32 masters
            emit_generic("tconv_compose",
                         lambda tname=tname, tf=tf: [self.master_ptr(tname + "/kernel"),
                                                     self.master_ptr(tf["consumer"] + "/kernel"), _ptr(tf["wg"])],
                         [tf["C"], tf["K"], tf["O"], tf["Ca"], tf["rs"]], [], "compose:" + tname)
        for li in range(len(layers) - 1, -1, -1):
            l = layers[li]
            if l.kind == "mask" and self._norm_head_loss:
                # head weight / bias gradients and the head input's norm-backward rows from
                # the forward's per-channel sums (no pass over the activation)
                hc = self.tinfo[self.head_in][1]
                Nb, Pb = self.B, self.npix(1) // self.B
                self._hn_rows = self._stat_buf("hn:rows", Nb * self.C.hn_blocks_per_sample(Nb, Pb) * 2 * hc)
                emit_generic("head_norm_coef",
                             lambda hc=hc: [_ptr(self._stat_bufs["hn:part"]), _ptr(self.sums),
                                            self.master_ptr("Mask/kernel"), _ptr(b["fa:" + self.head_in]),
                                            _ptr(b["fc:" + self.head_in]), _ptr(self._hn_rows),
                                            self.grad_ptr("Mask/kernel"), self.grad_ptr("Mask/bias"),
                                            _ptr(self.loss_scale_dev)],
                             [Nb, Pb, hc, 0 if spec.norm == "batch" else hc], [inv_total, self.bce_weight, 1.0],
                             "bwd:Mask")
                done("Mask")
            elif l.kind == "mask" and self.fusions.get("head_wsum"):
                if not self.head_onload:
                    # the head input's dY from its ReLU bits (the input was not stored)
                    hc = self.tinfo[self.head_in][1]
                    emit_generic("head_dy",
                                 lambda: [_ptr(self.relu_bits[self.head_in]), self.master_ptr("Mask/kernel"),
                                          _ptr(self.prob), _ptr(self.target), _ptr(self.sums),
                                          _ptr(b["d:" + self.head_in]), _ptr(self.loss_scale_dev)],
                                 [self.npix(1), hc], [inv_total, self.bce_weight, 1.0], "bwd:Mask")
                # the Mask gradients from the forward's per-workgroup sums (head_ws)
                emit_generic("head_wsum_grad",
                             lambda: [_ptr(self.head_ws), _ptr(self.sums), self.grad_ptr("Mask/kernel"),
                                      self.grad_ptr("Mask/bias"), _ptr(self.loss_scale_dev)],
                             [self._head_ws_rows], [inv_total, self.bce_weight, 1.0], "wgrad:Mask")
                done("Mask")
            elif l.kind == "mask":
                hc = self.tinfo[self.head_in][1]
                nb = self.head_nb
                # head-on-load: no dY is written, only the Mask gradients are reduced, off
                # the dgrad chain (side stream: "wgrad:" plan names)
                emit_generic("head_bwd",
                             lambda hc=hc: [_ptr(b[self.head_in]), self.master_ptr("Mask/kernel"), _ptr(self.prob),
                                            _ptr(self.target), _ptr(self.sums),
                                            0 if self.head_onload else _ptr(b["d:" + self.head_in]),
                                            _ptr(self.head_partial), self.grad_ptr("Mask/kernel"),
                                            self.grad_ptr("Mask/bias"), _ptr(self.loss_scale_dev)],
                             [P1, hc], [inv_total, self.bce_weight, 1.0],
                             "wgrad:Mask" if self.head_onload else "bwd:Mask")
                done("Mask")
            elif l.kind == "conv":
                src1, up1, skip = self.inputs[l.name]
                first = src1 == "x"
                c1 = self.tinfo[src1][1]
                c2 = self.tinfo[skip][1] if skip else 0
                onload = l.name == self.head_in and self.head_onload
                dy = self._no_dy if onload else b["d:" + l.name]
                first_xf = None
                if spec.norm != "none":
                    if first and self._fusion_ok("first_dz_onload"):
                        self._fusion_on("first_dz_onload", l.name)
                        # the first layer's dz is read only by its weight gradient: that kernel
                        # forms dz = ca g + cb z + cc on load (no norm_bwd_apply pass)
                        first_xf = dict(xform=2, xa=_ptr(b["ca:" + l.name]), xb=_ptr(b["cb:" + l.name]),
                                        xc=_ptr(b["cc:" + l.name]), xz=_ptr(b["z:" + l.name]),
                                        xcs=0 if spec.norm == "batch" else l.cout)
                    split_xf = None
                    if first_xf is None and not first:
                        split_xf = self._dz_split_fields(l, src1, skip)
                    ops.extend(self._norm_bwd_ops(l, apply=first_xf is None and split_xf is None))
                    dy = b["dz:" + l.name] if first_xf is None and split_xf is None else b["d:" + l.name]
                Q = self.npix(l.level)
                # --- weight + bias gradient (fused column sums); the upsampling decoder's
                # A operand is the materialised upsample when there is one
                wa_t = self._wa_chain_of.get(l.name)
                if wa_t is not None:
                    # chained u rows: the weight gradient runs over the skip source only;
                    # tconv_chain forms the u rows from H / Bs
                    a1, upA, c1w, c2w, skw = b[skip], 1, c2, 0, None
                    if self._skip_onload.get(skip) == l.name:
                        a1 = b["z:" + skip]          # (normalised on load: xform 1 below)
                else:
                    a1, upA, c1w, c2w, skw = (b[src1] if src1 in b else None), up1, c1, c2, skip
                if up1 == 2 and self.ups_materialize:
                    a1, upA = b["up:" + src1], 1
                kd = dict(N=self.B, QD=self.sdims(l.level)[0], QH=self.sdims(l.level)[1],
                          QW=self.sdims(l.level)[2], AD=self.sdims(l.level)[0], AH=self.sdims(l.level)[1],
                          AW=self.sdims(l.level)[2], KD=3 if self.dims == 3 else 1, KH=3, KW=3, stride=1,
                          pad=1, upA=upA, a1=_ptr(a1), a2=_ptr(b[skw]) if skw else None,
                          b=_ptr(dy))
                if first_xf is not None:
                    kd.update(first_xf)
                if spec.norm != "none" and split_xf is not None:
                    kd.update(split_xf)
                if wa_t is not None and self._skip_onload.get(skip) == l.name:
                    kd.update(xform=1, xa=_ptr(b["fa:" + skip]), xb=_ptr(b["fc:" + skip]),
                              xcs=0 if spec.norm == "batch" else self.tinfo[skip][1])
                if l.name == self.head_in and self.head_onload:
                    kd.update(self._head_grad_fields())
                wspec = dict(lname=l.name, kd=kd, M1=c1w, M2=c2w, Nc=l.cout, KT=KT3, Q=Q,
                             QD=self.sdims(l.level)[0], QH=self.sdims(l.level)[1],
                             QW=self.sdims(l.level)[2], upA=upA,
                             kernel=l.name + "/kernel", bias=l.name + "/bias", bias_mode=1,
                             bias_width=l.cout, bias_src=(dy, Q),
                             real_rows=(self.cpad, spec.in_channels) if first else None)
                if wa_t is not None:
                    wspec["kernel_out"] = _ptr(self.tconv_fused[wa_t]["wa"]["skg"])
                part_at = tail_parts.pop(l.name, None)
                if part_at is not None:
                    # first half of this weight gradient at the placeholder between the two
                    # halves of the consumer's dgrad, second half here
                    wspec["parts"] = 2
                    wg_specs.append(wspec)
                    ops[part_at] = ("wgrad", len(wg_specs) - 1, 0)
                    ops.append(("wgrad", len(wg_specs) - 1, 1))
                else:
                    emit_wgrad(wspec)
                # --- data gradient
                if not first:
                    def mk(l=l, src1=src1, up1=up1, skip=skip, c1=c1, c2=c2, dy=dy):
                        d = self._conv_common(l.level, 3, 1, 1)
                        d.update(name="dgrad:" + l.name, C1=l.cout, src1=_ptr(dy),
                                 wgt=self.wptr(l.name, "dg"), Cout=l.cin, relu=0)
                        if skip is None:
                            lvl, ch, relu_src, drop = self.tinfo[src1]
                            m1, mb = self._relu_mask(src1) if relu_src else (None, 0)
                            d.update(dst1=_ptr(b["d:" + src1]), D1=l.cin, mask1=m1, mask_bits=mb,
                                     mask_scale1=(1.0 / (1.0 - spec.dropout)) if drop else 1.0)
                            self._fuse_dgrad_norm(d, src1)
                            if l.name == self.head_in and self.head_onload:
                                d.update(self._head_grad_fields())
                        else:
                            dsk = self._skip_route(l, skip, c1, c2, dy)
                            tname = self._tf_consumer.get(l.name)
                            if tname is not None:
                                if dsk is None:
                                    raise RuntimeError("fused transposed conv %s: skip route of %s failed"
                                                       % (tname, l.name))
                                tf = self.tconv_fused[tname]
                                tsrc = tf["src"]
                                tl = next(x for x in spec.layers if x.name == tname)
                                d = self._conv_common(tl.level + 1, 3, 1, 1)
                                m1, mb = self._relu_mask(tsrc)
                                d.update(name="dgrad:" + l.name, C1=4 * l.cout, s2d=l.cout, src1=_ptr(dy),
                                         wgt=_ptr(tf["wg"]), Cout=tf["K"], relu=0, dst1=_ptr(b["d:" + tsrc]),
                                         D1=tf["K"], mask1=m1, mask_bits=mb)
                                self._fuse_dgrad_norm(d, tsrc)
                                if spec.norm != "none" and not d.get("nz"):
                                    raise RuntimeError("fused transposed conv %s: no dgrad-norm epilogue" % tname)
                                self._deferred_skip[dsk[0]] = dsk[1]
                                if spec.norm == "none":
                                    self._rev_order(d, "g:" + l.name, "g:" + tsrc)
                                return d
                            if up1 == 2:
                                dst1 = b["dfull:" + src1]          # full-res grad of the upsample
                            else:
                                dst1 = b["d:" + src1]              # tconv output: linear, no mask
                            if dsk is not None:
                                # the skip half runs later, fused with the pool backward
                                d.update(Cout=c1, dst1=_ptr(dst1), D1=c1)
                                self._deferred_skip[dsk[0]] = dsk[1]
                            else:
                                m2, mb = self._relu_mask(skip)
                                d.update(dst1=_ptr(dst1), D1=c1, dst2=_ptr(b["dskip:" + skip]),
                                         mask2=m2, mask_bits=2 * mb)
                        if spec.norm == "none":
                            self._rev_order(d, "g:" + l.name, "g:" + src1)
                        return d
                    dd_ = mk()                 # built now: it decides the fused norm backward
                    if spec.norm != "none" and split_xf is not None:
                        dd_.update(split_xf)
                    halves = self._tail_halves(dd_, l, src1, skip, dy)
                    parts = self._plan_dw_fuse(l, src1, skip, [dd_] if halves is None else list(halves), wspec)
                    if parts is not None:
                        halves = None if len(parts) == 1 else parts
                        dd_ = parts[0]

                    def fin(h, w=wspec):
                        # fused weight gradient: the slab rows of this layer's weight-gradient spec
                        return dict(h, fw_slab=w["slab_ptrs"][0], fw_bias_slab=w["slab_ptrs"][1]) if "dw" in w else h
                    if halves is None:
                        emit_conv(lambda dd_=dd_, fin=fin: fin(dd_))
                    else:
                        # the last dgrad of the chain in two batch halves: the first layer's
                        # weight gradient (the backward's tail, alone on the GPU otherwise)
                        # starts on the side stream as soon as the first half is written
                        emit_conv(lambda h=halves[0], fin=fin: fin(h))
                        tail_parts[src1] = len(ops)
                        ops.append(("placeholder",))
                        emit_conv(lambda h=halves[1], fin=fin: fin(h))
                    if up1 == 2:
                        lvl = self.tinfo[src1][0]
                        dd, hh, ww = self.sdims(lvl)
                        emit_generic("ups_bwd",
                                     lambda src1=src1: [_ptr(b["dfull:" + src1]), _ptr(b[src1]),
                                                        _ptr(b["d:" + src1])],
                                     [self.B, dd, hh, ww, c1, int(self.dims == 3)], [], "bwd:up:" + src1)
                done(l.name)
            elif l.kind == "pool" and l.name in self._deferred_skip:
                # the decoder conv's skip-half data gradient with this pool's backward
                # in its epilogue: writes d:<convNb> in one pass
                emit_conv(lambda dsk=self._deferred_skip[l.name]: dsk)
            elif l.kind == "pool" and src_normed(self.inputs[l.name][0]):
                # gradient of a normalised convNb output: the pool backward also emits
                # the norm's backward statistics (no separate nstat_bwd pass)
                src = self.inputs[l.name][0]
                dd, hh, ww = self.sdims(l.level)
                P_ = self.npix(l.level + 1) // self.B
                nbp = self.C.norm_blocks_per_sample(self.B, P_)
                rows = self._stat_buf("bst:" + src, self.B * nbp * 2 * l.cout)
                self._bwd_fused[src] = (self.B * nbp, True)
                emit_generic("pool_bwd_norm",
                             lambda src=src, l=l, rows=rows: [
                                 _ptr(self.pool_codes[l.name]), _ptr(b["d:" + l.name]),
                                 _ptr(b["dskip:" + src]) if ("dskip:" + src) in b else 0,
                                 _ptr(b["z:" + src]), _ptr(b["d:" + src]), _ptr(rows)],
                             [self.B, dd, hh, ww, l.cout, int(self.dims == 3), nbp], [], "bwd:" + l.name)
            elif l.kind == "pool":
                src = self.inputs[l.name][0]
                dd, hh, ww = self.sdims(l.level)
                emit_generic("pool_bwd",
                             lambda src=src, l=l: [_ptr(b[src]), _ptr(b["d:" + l.name]),
                                                   _ptr(b["dskip:" + src]) if ("dskip:" + src) in b else 0,
                                                   _ptr(b["d:" + src]), _ptr(self.pool_codes[l.name])],
                             [self.B, dd, hh, ww, l.cout, int(self.dims == 3)], [], "bwd:" + l.name)
            elif l.kind == "tconv" and l.name in self.tconv_fused:
                tf = self.tconv_fused[l.name]
                lo, hi = self.sdims(l.level + 1), self.sdims(l.level)
                # the consumer's pre-activation gradient (its norm backward's dz when normalised)
                dz = b[("dz:" if spec.norm != "none" else "d:") + tf["consumer"]]
                kd = dict(N=self.B, QD=1, QH=lo[1], QW=lo[2], AD=1, AH=hi[1], AW=hi[2], KD=1, KH=4, KW=4,
                          stride=2, pad=1, upA=1, a1=_ptr(dz), b=_ptr(b[tf["src"]]))
                emit_wgrad(dict(lname=l.name, kd=kd, M1=tf["O"], M2=0, Nc=tf["K"], KT=16, QW=lo[2],
                                Q=self.npix(l.level + 1), kernel=None, kernel_out=_ptr(tf["hs"]),
                                bias=None, bias_out=_ptr(tf["bs"]), bias_mode=2, bias_width=16 * tf["O"],
                                bias_per_tap=True, real_rows=None, bias_src=(dz, self.npix(l.level + 1)),
                                chain=l.name))
                done(l.name)
            elif l.kind == "tconv":
                src = self.inputs[l.name][0]
                du = b["d:" + l.name]
                lo = self.sdims(l.level + 1)
                hi = self.sdims(l.level)
                kd = dict(N=self.B, QD=lo[0], QH=lo[1], QW=lo[2], AD=hi[0], AH=hi[1], AW=hi[2],
                          KD=2 if self.dims == 3 else 1, KH=2, KW=2, stride=2, pad=0, upA=1,
                          a1=_ptr(du), b=_ptr(b[src]))
                emit_wgrad(dict(lname=l.name, kd=kd, M1=l.cout, M2=0, Nc=l.cin, KT=KT2,
                                QW=lo[2] if self.dims == 2 else 0,
                                Q=self.npix(l.level + 1), kernel=l.name + "/kernel",
                                bias=l.name + "/bias", bias_mode=2, bias_width=l.cout, real_rows=None,
                                bias_src=(du, self.npix(l.level))))

                def mk(l=l, src=src, du=du):
                    d = self._conv_common(l.level + 1, 2, 2, 0, out_level=l.level + 1, in_level=l.level)
                    m1, mb = self._relu_mask(src)
                    d.update(name="dgrad:" + l.name, C1=l.cout, src1=_ptr(du),
                             wgt=self.wptr(l.name, "dg"), Cout=l.cin, relu=0,
                             dst1=_ptr(b["d:" + src]), mask1=m1, mask_bits=mb)
                    self._fuse_dgrad_norm(d, src)
                    return d
                dd_ = mk()
                emit_conv(lambda dd_=dd_: dd_)
                done(l.name)
            elif l.kind == "up":
                pass

        # size the wgrad workspaces: every wgrad gets its own slab / bias-slab / stage
        # region (HBM is plentiful) so the split-K reductions of several layers can be
        # batched into one launch per phase (multi_reduce), flushed every few layers
        sized = [self._wgrad_splits(w) for w in wg_specs]
        for k, w in enumerate(wg_specs):
            if w.get("parts"):                     # each half keeps the full grid
                sp = sized[k]
                sized[k] = (2 * sp[0],) + tuple(sp[1:])
            if "dw" in w:                          # fused into the data gradient: its slab rows
                sized[k] = (w["dw"]["rows"], w["M1"], KT3, 1, 0)
        stot = btot = sttot = 0
        regions = []
        for w, (splits, Mtot, taps, tg, smallc) in zip(wg_specs, sized):
            bw = w["bias_width"] if w["bias_mode"] == 1 else Mtot
            ncol = self._colsum_blocks(w["bias_src"][1], w["bias_width"])
            nb_rows = max(splits * tg, ncol)
            st_k = self.C.reduce_groups(splits) * taps * Mtot * w["Nc"]
            st_b = self.C.reduce_groups(nb_rows) * max(bw, w["bias_width"])
            regions.append((stot, btot, sttot, sttot + _r64(st_k)))
            stot += _r64(splits * taps * Mtot * w["Nc"])
            btot += _r64(nb_rows * max(bw, w["bias_width"]))
            sttot += _r64(st_k) + _r64(st_b)
        self.slab = torch.empty(max(stot, 64), dtype=torch.float32, device=self.device)
        self.bias_slab = torch.empty(max(btot, 64), dtype=torch.float32, device=self.device)
        self.red_stage = torch.empty(max(sttot, 64), dtype=torch.float32, device=self.device)
        self._job_tables = []
        job_dt = np.dtype([("slab", "<i8"), ("out", "<i8"), ("stage", "<i8"), ("n4", "<i8"), ("n4o", "<i8"),
                           ("p1", "<i8"), ("p2", "<i8"), ("splits", "<i4"), ("groups", "<i4"), ("taps", "<i4"),
                           ("Mtot", "<i4"), ("Mout", "<i4"), ("Nc", "<i4"), ("rg", "<i4"), ("rkeep", "<i4"),
                           ("direct", "<i4"), ("pad", "<i4")])
        assert job_dt.itemsize == self.C.reduce_job_bytes()
        pending_jobs, pending_layers = [], []
        pending_tags = []            # reduced here but complete only after a later chain rule
        wgrad_layers = {w["lname"] for w in wg_specs}
        FLUSH_LAYERS = 3

        def job(slab, out, stage, splits, taps, Mtot, Mout, Nc, rg=0, rkeep=0):
            rg = rg if rg > 0 else Mout
            rkeep = rkeep if rkeep > 0 else rg
            groups = self.C.reduce_groups(splits)
            direct = int(groups == 1 and Mout == Mtot and rg == rkeep)
            assert (taps * Mtot * Nc) % 4 == 0 and (taps * Mout * Nc) % 4 == 0
            return dict(slab=slab, out=out, stage=stage, n4=taps * Mtot * Nc // 4, n4o=taps * Mout * Nc // 4,
                        splits=splits, groups=groups, taps=taps, Mtot=Mtot, Mout=Mout, Nc=Nc, rg=rg, rkeep=rkeep,
                        direct=direct)

        def flush():
            if not pending_jobs:
                return
            arr = np.zeros(len(pending_jobs), dtype=job_dt)
            t1 = t2 = 0
            for k, j in enumerate(pending_jobs):
                for f in ("slab", "out", "stage", "n4", "n4o", "splits", "groups", "taps", "Mtot", "Mout", "Nc",
                          "rg", "rkeep", "direct"):
                    arr[k][f] = j[f]
                arr[k]["p1"], arr[k]["p2"] = t1, t2
                # (ranges padded to whole 256-thread blocks: block-uniform job lookup)
                t1 += -(-j["groups"] * j["n4"] // 256) * 256
                t2 += 0 if j["direct"] else -(-j["n4o"] // 256) * 256
            table = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)
            self._job_tables.append(table)
            plan.add_generic("multi_reduce", [_ptr(table)], [len(pending_jobs), t1, t2], [],
                             "reduce:" + ",".join(pending_layers + pending_tags))
            # (the stage is written by the op's phase 1 and read by its phase 2)
            plan.annotate(reads=[j["slab"] for j in pending_jobs],
                          writes=[j["out"] for j in pending_jobs] +
                          [j["stage"] for j in pending_jobs if not j["direct"]])
            for ln in pending_layers:
                self._layer_done_at[ln] = plan.size()
            pending_jobs.clear()
            pending_layers.clear()
            pending_tags.clear()

        slab0, bslab0, stage0 = _ptr(self.slab), _ptr(self.bias_slab), _ptr(self.red_stage)
        # layers whose gradients are complete only after a chain rule (a fused tconv; the
        # consumer of a composite forward, whose u rows the chain writes)
        chained = set(self._wa_chain_of)
        for op in ops:
            if callable(op):
                op(plan)
            elif op[0] == "done":
                if op[1] in chained:
                    if op[1] in self._wa_chain_of:  # done after its chain rule
                        pending_tags.append(op[1])
                elif op[1] in wgrad_layers:
                    pending_layers.append(op[1])
                    if len(pending_layers) >= FLUSH_LAYERS:
                        flush()
                else:
                    self._layer_done_at[op[1]] = plan.size()
            elif op[0] == "wgrad":
                w = wg_specs[op[1]]
                part = op[2] if len(op) > 2 else None
                splits, Mtot, taps, tg, smallc = sized[op[1]]
                so, bo, sto_k, sto_b = regions[op[1]]
                slab, bslab = slab0 + 4 * so, bslab0 + 4 * bo
                stage_k, stage_b = stage0 + 4 * sto_k, stage0 + 4 * sto_b
                d = dict(w["kd"])
                BM = self._wgrad_pick(w)[0]
                # the 128x128 tile has no register room for the fused ones-MFMA bias sums:
                # those (level >= 3, small dY) use a separate column-sum pass instead
                fused_bias = BM < 128
                if w["lname"] == self.head_in and self.head_onload and not fused_bias:
                    raise RuntimeError("head-on-load: the head input's weight gradient needs the fused-bias "
                                       "tile (its dY is never materialised for a column-sum pass)")
                d.update(name="wgrad:" + w["lname"], M1=w["M1"], M2=w["M2"], Nc=w["Nc"], splits=splits,
                         win=self.wgrad_win, slab=slab, bias_mode=w["bias_mode"] if fused_bias else 0,
                         bias_slab=bslab, pair=int(self.opts["wg_pair"] >= (1 if self.dims == 3 else 2)),
                         pf=int(self.opts["wg_pf"] >= (1 if self.dims == 3 else 2) or d.get("xform") == 1))
                if part is not None:
                    d.update(split_lo=part * splits // 2, split_n=splits // 2)
                if "dw" in w:
                    # computed by the fused data-gradient launch(es) that follow in the plan;
                    # only the slab reduction is planned here
                    w["slab_ptrs"] = (slab, bslab)
                else:
                    self._add_wgrad_chunked(plan, d, taps * Mtot * w["Nc"],
                                            (w["bias_width"] if w["bias_mode"] == 1 else Mtot) * tg)
                if part == 0:
                    continue                       # the reductions follow the last part
                KT = w["KT"]
                kout = w.get("kernel_out") or self.grad_ptr(w["kernel"])
                bout = w.get("bias_out") or self.grad_ptr(w["bias"])
                if smallc:
                    cpad, creal = w["real_rows"]
                    pending_jobs.append(job(slab, kout, stage_k, splits, 1, Mtot, KT * creal, w["Nc"], cpad, creal))
                else:
                    pending_jobs.append(job(slab, kout, stage_k, splits, taps, Mtot, Mtot, w["Nc"]))
                bw = w["bias_width"]
                if not fused_bias:
                    src, rows = w["bias_src"]
                    nb = self._colsum_blocks(rows, bw)
                    plan.add_generic("colsum", [_ptr(src), bslab], [rows, bw, nb], [], "bsum:" + w["lname"])
                    pending_jobs.append(job(bslab, bout, stage_b, nb, 1, 1, 1, bw))
                elif w["bias_mode"] == 1:
                    pending_jobs.append(job(bslab, bout, stage_b, splits, 1, 1, 1, bw))
                elif w.get("bias_per_tap"):
                    # [splits][tg][Mtot] rows -> per-tap sums [tg][Mtot]
                    pending_jobs.append(job(bslab, bout, stage_b, splits, 1, 1, 1, bw))
                else:
                    # [splits*tg][Mtot] rows -> bias (Mtot == cout for tconv)
                    pending_jobs.append(job(bslab, bout, stage_b, splits * tg, 1, 1, 1, bw))
                if w.get("chain"):
                    # the slab sums are reduced now; the chain rule writes the tconv gradients
                    tname = w["chain"]
                    tf = self.tconv_fused[tname]
                    pending_layers.append(tname)
                    flush()
                    chained.add(tname)
                    ptrs = [_ptr(tf["hs"]), _ptr(tf["bs"]), self.master_ptr(tf["consumer"] + "/kernel"),
                            self.grad_ptr(tname + "/kernel"), self.grad_ptr(tname + "/bias")]
                    sf = tf.get("wa")
                    if sf is not None:
                        # + the consumer's weight gradient: u rows from H / Bs, skip rows copied
                        assert tf["consumer"] not in pending_layers
                        ptrs += [self.master_ptr(tname + "/kernel"), self.master_ptr(tname + "/bias"),
                                 _ptr(sf["skg"]), self.grad_ptr(tf["consumer"] + "/kernel")]
                    plan.add_generic("tconv_chain", ptrs, [tf["C"], tf["K"], tf["O"], tf["Ca"]], [], "chain:" + tname)
                    self._layer_done_at[tname] = plan.size()
                    if sf is not None:
                        self._layer_done_at[tf["consumer"]] = plan.size()
        flush()
        for name in self._dz_onload:
            # formed on load by the fused data + weight gradient: never stored (kept aside so
            # the plan validation flags any op that would still read it)
            self._dropped["dz:" + name] = self.bufs.pop("dz:" + name, None)

    def _add_wgrad_chunked(self, plan, d, row_floats, brow_floats):
        """plan.add_wgrad(d); a tiled (non-window) weight gradient whose operand tensors
        exceed the 2 GiB reach of one 32-bit buffer base (3D 128^3 at 16 volumes, 512^2 at 128
        images: the first layer's) runs as batch chunks instead -- chunk k takes images
        [k N / c, (k + 1) N / c) and slab rows [k S / c, (k + 1) S / c) of the same slabs, so
        the fixed-order reduction is unchanged."""
        try:
            return plan.add_wgrad(d)
        except ValueError as ex:
            if "2 GiB" not in str(ex) or d.get("xform") or d.get("hg_prob") or d.get("split_n") or d.get("upA", 1) != 1:
                raise
        N, S = d["N"], d["splits"]
        a_img = d.get("AD", 1) * d.get("AH", 1) * d.get("AW", 1) * 2
        b_img = d.get("QD", 1) * d.get("QH", 1) * d.get("QW", 1) * d["Nc"] * 2
        lim = (1 << 31) - 64
        per = max(a_img * max(d["M1"], d.get("M2") or 0), b_img)
        c = 2
        while (N + c - 1) // c * per >= lim:
            c += 1
        if c > min(N, S):
            raise ValueError("wgrad: cannot chunk the batch under the 2 GiB buffer reach")
        for k in range(c):
            n0, n1 = k * N // c, (k + 1) * N // c
            s0, s1 = k * S // c, (k + 1) * S // c
            dk = dict(d, N=n1 - n0, splits=s1 - s0, a1=d["a1"] + n0 * a_img * d["M1"],
                      b=d["b"] + n0 * b_img, slab=d["slab"] + 4 * s0 * row_floats)
            if d.get("a2"):
                dk["a2"] = d["a2"] + n0 * a_img * d["M2"]
            if d.get("bias_mode"):
                dk["bias_slab"] = d["bias_slab"] + 4 * s0 * brow_floats
            plan.add_wgrad(dk)

    # ------------------------------------------------------------------ buckets
    def set_buckets(self, bounds: Optional[Sequence[int]]):
        """bounds: flat-buffer element offsets ending each allreduce bucket.  A
        segment ends at the first plan op after which every layer whose
        variables lie below the bound has finished its gradient."""
        self.seg_ends = []
        self.seg_bounds = []
        if not bounds:
            self.seg_ends = [self.bwd_end]
            self.seg_bounds = [self.flat.numel]
            return
        for bound in bounds:
            last = self.fwd_end
            for name, shape, off, n in self.flat.entries:
                if off < bound:
                    last = max(last, self._layer_done_at[name.split("/")[0]])
            self.seg_ends.append(last)
            self.seg_bounds.append(bound)
        self.seg_ends[-1] = self.bwd_end

    # ------------------------------------------------------------------ running
    def load_batch(self, x: torch.Tensor, y: torch.Tensor, stream=None):
        """x: [B, (D,) H, W, Cin] float, y: [B, (D,) H, W, 1] float/bool."""
        cin = self.spec.in_channels
        if (x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32 and x.is_contiguous()
                and y.is_contiguous() and x.shape[0] == self.B and y.numel() * cin == x.numel()):
            # one launch: cast into the channel-padded 16-bit input and the target
            if getattr(self, "_iota", None) is None:
                self._iota = torch.arange(self.B, device=self.device, dtype=torch.int64)
            return self.load_indexed(x, y, self._iota, stream)
        xb = self.bufs["x"].view(-1, self.cpad)
        (xb if cin == self.cpad else xb[:, :cin]).copy_(x.reshape(-1, cin), non_blocking=True)
        self.target.copy_(y.reshape(-1), non_blocking=True)

    def load_indexed(self, x_all: torch.Tensor, y_all: torch.Tensor, idx: torch.Tensor, stream=None):
        """Batch = samples `idx` (device int64) of the HBM-resident dataset, gathered
        and cast straight into the padded 16-bit input and target (one launch)."""
        cin = self.spec.in_channels
        P = x_all[0].numel() // cin
        assert idx.dtype == torch.int64 and idx.numel() == self.B and x_all.dtype == torch.float32
        assert y_all[0].numel() == P and x_all.is_contiguous() and y_all.is_contiguous()
        self.C.generic("gather_batch", [_ptr(x_all), _ptr(y_all), _ptr(idx), _ptr(self.bufs["x"]), _ptr(self.target)],
                       [self.B, P, cin, self.cpad], [], native.stream_handle(stream), self.dt_id)

    # ------------------------------------------------------------------ HIP graphs
    def enable_graphs(self):
        """Replay the forward, every backward segment and the Adam launch as captured
        HIP graphs (one graph launch instead of ~150 kernel launches per step).

        Values that change per step live in device memory so the frozen kernel
        arguments stay valid: the dropout seed (``Plan.set_seed_ptr``) and Adam's
        {lr_t, grad scale}.  Segments are captured separately so the bucketed
        allreduces still start eagerly between segment replays (overlap unchanged).
        Graphs are captured lazily on first use and dropped when buckets change."""
        if self.device.type != "cuda":
            raise RuntimeError("HIP graphs need a GPU")
        self.seed_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.adam_scalars = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.plan.set_seed_ptr(_ptr(self.seed_dev))
        self.graphs = {}

    def _replay(self, key, launch):
        g = self.graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                launch(native.stream_handle(None))
            self.graphs[key] = g
        g.replay()

    def set_loss_scale(self, scale: float):
        """Scale of the loss gradient entering the backward (all parameter gradients
        scale with it); lives on the device so plans and graphs need no rebuild."""
        if scale != self._loss_scale:
            self.loss_scale_dev.fill_(scale)
            self._loss_scale = scale

    def _forward_2s(self, stream):
        """Chunk 0 on the caller's stream; chunk 1 on a side stream once chunk 0 has
        finished its first layers; the head finish after both."""
        main = stream if stream is not None else torch.cuda.current_stream()
        if getattr(self, "_fside", None) is None:
            self._fside = torch.cuda.Stream(device=self.device)
            self._fev = torch.cuda.Event()
        side = self._fside
        (a0, m0, e0), (a1, m1, e1) = self._fwd2
        hm, hs = main.cuda_stream, side.cuda_stream
        side.wait_stream(main)                      # inputs loaded, previous step done
        self.plan.run(a0, m0, hm)
        self._fev.record(main)
        self.plan.run(m0, e0, hm)
        side.wait_event(self._fev)
        self.plan.run(a1, e1, hs)
        main.wait_stream(side)
        self.plan.run(e1, self.fwd_end, hm)

    def forward(self, seed: int, stream=None):
        seed &= 0xFFFFFFFF
        self.plan.set_seed(seed)
        if getattr(self, "_fwd2", None) is not None and self._fwd_streams(True) == 2:
            if self.graphs is not None:
                self.seed_dev.fill_(seed - (1 << 32) if seed >= (1 << 31) else seed)
            return self._forward_2s(stream)
        if self.graphs is not None:
            self.seed_dev.fill_(seed - (1 << 32) if seed >= (1 << 31) else seed)
            with torch.cuda.stream(stream) if stream is not None else _nullctx():
                self._replay(("fwd", self.fwd_end), lambda s: self.plan.run(0, self.fwd_end, s))
            return
        self.plan.run(0, self.fwd_end, native.stream_handle(stream))

    _SIDE_KINDS = ("wgrad:", "bsum:", "reduce:", "chain:")

    def _side_groups(self, begin, end):
        """[begin, end) as maximal runs of (on_side, i, j): weight-gradient launches
        on the side stream, everything else on the main stream."""
        key = (begin, end)
        g = self._groups.get(key)
        if g is None:
            names = self.plan.names()
            g = []
            i = begin
            while i < end:
                side = names[i].startswith(self._SIDE_KINDS)
                j = i
                while j < end and names[j].startswith(self._SIDE_KINDS) == side:
                    j += 1
                g.append((side, i, j))
                i = j
            self._groups[key] = g
        return g

    def _backward_dual(self, on_segment, stream):
        """Eager backward with the weight gradients on a side stream.  Every side run
        first waits for all dgrad-chain work enqueued so far (its dY and any earlier
        gradient producers); bucket allreduces are issued from the side stream after
        it has also caught up with the chain, so the dgrad chain never waits for them;
        the caller's stream joins both at the end (the next forward overwrites
        activations the side launches read).  (Stream priorities for either chain
        measured no effect in round 2.)"""
        main = stream if stream is not None else torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        chain = main
        side = self._side
        hm, hs = chain.cuda_stream, side.cuda_stream
        begin = self.fwd_end
        for k, end in enumerate(self.seg_ends):
            for on_side, i, j in self._side_groups(begin, end):
                if on_side:
                    side.wait_stream(chain)
                    self.plan.run(i, j, hs)
                else:
                    self.plan.run(i, j, hm)
            begin = end
            if on_segment is not None:
                side.wait_stream(chain)
                with torch.cuda.stream(side):
                    on_segment(k)
        main.wait_stream(side)

    def backward(self, on_segment=None, stream=None):
        if self.dual_stream and self.device.type == "cuda":
            return self._backward_dual(on_segment, stream)
        s = native.stream_handle(stream)
        begin = self.fwd_end
        for i, end in enumerate(self.seg_ends):
            if end == begin:
                pass                    # bucket finished by the previous segment already
            elif self.graphs is not None:
                with torch.cuda.stream(stream) if stream is not None else _nullctx():
                    self._replay(("bwd", begin, end), lambda hs, b=begin, e=end: self.plan.run(b, e, hs))
            else:
                self.plan.run(begin, end, s)
            begin = end
            if on_segment is not None:
                on_segment(i)

    def evaluate_batch(self, stream=None):
        """Inference forward (eval plan) of the loaded batch; sums -> self.sums."""
        self.eval_plan.set_seed(0)
        self.eval_plan.run(0, self.eval_plan.size(), native.stream_handle(stream))

    def probs(self) -> torch.Tensor:
        d, h, w = self.sdims(1)
        shape = (self.B, h, w, 1) if self.dims == 2 else (self.B, d, h, w, 1)
        return self.prob.view(shape)
