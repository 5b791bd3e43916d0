"""Static validation of the native executor's launch plans (no GPU needed).

The planner (`runtime/native_engine.py`) decides a dozen cross-layer fusions whose
legality depends on the config (norm x decoder x dims x image size).  A wrong decision
shows up either as a launch whose parameters no built kernel accepts, or as a kernel
reading a buffer nothing wrote in that step (silently stale data).  This module checks
both on a dry-run plan:

* **dispatch** -- every op of the training and evaluation plans is run through its
  launcher under dry dispatch (`Plan.check_dispatch`, conv_params.h `dry_dispatch`): the
  launcher resolves its template instantiation / tile / epilogue and reports whether a
  kernel exists, without launching;
* **def-use** -- the executor records each op's parameters (`RecordingPlan`); every
  pointer an op reads must lie in a buffer that an EARLIER op of the same plan wrote, or
  in a step input (the batch, the weights, the running statistics, workspaces); pointers
  into no known buffer, and buffers the planner dropped (never formed), are errors;
* **coverage** -- every parameter's gradient (per variable of the flat buffer) is
  written by the training plan.

The reference has no such machinery (its graph is TF's, `test_dist.py:183-298`); this is
the static-graph executor's equivalent of TF's graph validation.
"""

from typing import Dict, List, Tuple

import torch

_HG = ("hg_prob", "hg_t", "hg_sums", "hg_w", "hg_bits", "hg_gscale", "hg_fa", "hg_fc")
CONV_READS = ("src1", "src2", "wgt", "bias", "mask1", "mask2", "route_gy", "nz", "na", "nc", "xa", "xb", "xc", "xz",
              "ut_x", "ut_w", "ut_b", "head_w", "head_b", "head_t", "fw_x") + _HG
CONV_WRITES = ("dst1", "dst2", "stats", "relu_bits", "pool_dst", "head_logit", "head_ws", "xout", "fw_slab",
               "fw_bias_slab")
WGRAD_READS = ("a1", "a2", "b", "xa", "xb", "xc", "xz") + _HG
WGRAD_WRITES = ("slab", "bias_slab")


def _sel(p, idx):
    return [p[i] for i in idx if i < len(p)]


def _conv_write_spans(d, stat_tiles=None) -> List[Tuple[int, int]]:
    """(pointer, bytes) of the writes of 16-bit conv dict `d` whose extent follows from its
    shape (the executor's offset arithmetic -- batch chunks, tail halves, channel splits,
    slab rows -- must keep each inside its buffer)."""
    g = d.get
    N, OD, OH, OW = g("N", 1), g("OD", 1) or 1, g("OH", 1), g("OW", 1)
    M = N * OD * OH * OW
    Cout = g("Cout", 0)
    D1 = g("D1") or Cout
    out = []
    if g("shuffle"):
        out.append((g("dst1"), M * Cout * 2))
    else:
        out.append((g("dst1"), M * D1 * 2))
        if g("dst2"):
            out.append((g("dst2"), M * (Cout - D1) * 2))
    if g("relu_bits"):
        out.append((g("relu_bits"), M * Cout // 8))
    if g("head_logit"):
        out.append((g("head_logit"), M * 4))
    if g("head_ws"):
        out.append((g("head_ws"), g("head_ws_rows", 0) * 100 * 4))
    if g("pool_dst"):
        out.append((g("pool_dst"), M // 4 * Cout * 2))
        out.append((g("pool_code"), M // 4 * Cout // 8 * 4))
    if g("xout"):
        out.append((g("xout"), M * g("C1", 0) * 2))
    if g("fw_x"):
        rows = g("fw_split_lo", 0) + g("fw_nsplit", 0)
        out.append((g("fw_slab"), rows * 9 * g("fw_Cx", 0) * g("C1", 0) * 4))
        out.append((g("fw_bias_slab"), rows * g("C1", 0) * 4))
    if g("stats") and stat_tiles is not None:
        rows = stat_tiles(d)
        if rows:
            out.append((g("stats"), rows * 2 * Cout * 4))
    return [(p, n) for p, n in out if p]


def _generic_write_spans(kind: str, p: List[int], ints: List[int]) -> List[Tuple[int, int]]:
    """(pointer, bytes) of the writes of the streaming norm passes (N, P, C in ints) and
    the head dY pass (P, C)."""
    if kind in ("norm_apply", "norm_bwd_apply") and len(p) > 5 and len(ints) >= 3:
        return [(p[5], ints[0] * ints[1] * ints[2] * 2)]
    if kind == "head_dy" and len(p) > 5 and len(ints) >= 2:
        return [(p[5], ints[0] * ints[1] * 2)]
    return []


def _generic_rw(kind: str, p: List[int], ints: List[int]) -> Tuple[List[int], List[int]]:
    """(read pointers, written pointers) of one generic op (layouts: bindings.cpp)."""
    if kind == "ups_fwd":
        return _sel(p, [0]), _sel(p, [1])
    if kind == "ups_bwd":
        return _sel(p, [0, 1]), _sel(p, [2])
    if kind == "pool_fwd":
        return _sel(p, [0]), _sel(p, [1, 2])
    if kind == "pool_bwd":
        return (_sel(p, [1, 2, 4]) if len(p) > 4 and p[4] else _sel(p, [0, 1, 2])), _sel(p, [3])
    if kind == "pool_bwd_norm":
        return _sel(p, [0, 1, 2, 3]), _sel(p, [4, 5])
    if kind == "norm_pool":
        return _sel(p, [0, 1, 2]), _sel(p, [3, 4, 5])
    if kind == "norm_apply" or kind == "norm_bwd_apply":
        return _sel(p, [0, 1, 2, 3, 4]), _sel(p, [5])
    if kind == "norm_rows":
        return _sel(p, [0, 1]), _sel(p, [2])
    if kind == "bn_stats":
        mode = ints[2]
        if mode == 0:
            return _sel(p, [0, 1, 2, 3, 4, 14]), _sel(p, [3, 4, 5, 6, 7, 8, 14])
        if mode == 1:
            return _sel(p, [0, 1, 2, 5, 6, 14]), _sel(p, [9, 10, 11, 12, 13, 14])
        return _sel(p, [1, 2, 3, 4]), _sel(p, [5, 6, 7, 8])
    if kind == "gn_stats":
        if ints[5] == 0:
            return _sel(p, [0, 1, 2]), _sel(p, [3, 4, 5, 6, 12])
        return _sel(p, [0, 1, 3, 4, 12]), _sel(p, [7, 8, 9, 10, 11, 12])
    if kind == "head_finish":
        return _sel(p, [0, 1]), _sel(p, [0, 2, 3])
    if kind == "head_fwd":
        return _sel(p, [0, 1, 2, 3]), _sel(p, [4, 5, 6])
    if kind == "head_wsum_grad":
        return _sel(p, [0, 1, 4]), _sel(p, [2, 3])
    if kind == "head_dy":
        return _sel(p, [0, 1, 2, 3, 4, 6]), _sel(p, [5])
    if kind == "head_bwd":
        return _sel(p, [0, 1, 2, 3, 4, 9]), _sel(p, [5, 6, 7, 8])
    if kind == "norm_head":
        return _sel(p, [0, 1, 2, 3, 4]), _sel(p, [5, 6])
    if kind == "norm_head_loss":
        return _sel(p, [0, 1, 2, 3, 4, 5]), _sel(p, [6, 7, 8, 9])
    if kind == "head_norm_coef":
        return _sel(p, [0, 1, 2, 3, 4, 8]), _sel(p, [5, 6, 7])
    if kind == "head_norm_bwd":
        return _sel(p, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11]), _sel(p, [10])
    if kind == "colsum":
        return _sel(p, [0]), _sel(p, [1])
    if kind == "tconv_compose":
        return _sel(p, [0, 1]), _sel(p, [2])
    if kind == "tconv_chain":
        return _sel(p, [0, 1, 2, 5, 6, 7]), _sel(p, [3, 4, 8])
    if kind == "wgrad_reduce":
        return _sel(p, [0]), _sel(p, [1, 2])
    if kind in ("f32_pool_fwd", "f32_ups_fwd", "f32_transpose"):
        return _sel(p, [0]), _sel(p, [1])
    if kind == "f32_pool_bwd":
        return _sel(p, [0, 1, 2]), _sel(p, [3])
    if kind == "f32_ups_bwd":
        return _sel(p, [0, 1]), _sel(p, [2])
    if kind == "f32_head_fwd":
        return _sel(p, [0, 1, 2, 3]), _sel(p, [4, 5, 6])
    if kind == "f32_head_bwd":
        return _sel(p, [0, 1, 2, 3, 4]), _sel(p, [5, 6, 7, 8])
    if kind == "f32_colsum":
        return _sel(p, [0]), _sel(p, [1, 2])
    if kind == "multi_reduce":
        return _sel(p, [0]), []          # slab / out pointers: the op's annotation (RecordingPlan.annotate)
    raise KeyError("plan_check: no read/write layout for generic op %r" % kind)


class RecordingPlan:
    """A native `_C.Plan` that also keeps each op's parameters for `check_plan`."""

    def __init__(self, plan, stat_tiles=None):
        self._plan = plan
        self._stat_tiles = stat_tiles        # conv dict -> statistics rows (extent of `stats`)
        self.ops: List[dict] = []

    def add_conv_fwd(self, d):
        i = self._plan.add_conv_fwd(d)
        reads = [d.get(k) for k in CONV_READS]
        writes = [d.get(k) for k in CONV_WRITES]
        (reads if d.get("route_gy") else writes).append(d.get("pool_code"))
        self.ops.append(dict(name=d.get("name", "conv_fwd"), reads=reads, writes=writes,
                             spans=_conv_write_spans(d, self._stat_tiles)))
        return i

    def add_wgrad(self, d):
        i = self._plan.add_wgrad(d)
        self.ops.append(dict(name=d.get("name", "wgrad"), reads=[d.get(k) for k in WGRAD_READS],
                             writes=[d.get(k) for k in WGRAD_WRITES]))
        return i

    def add_f32_conv(self, d):
        i = self._plan.add_f32_conv(d)
        self.ops.append(dict(name=d.get("name", "f32_conv"), reads=[d.get(k) for k in ("src1", "src2", "wgt", "bias",
                                                                                        "mask1")],
                             writes=[d.get("dst1")]))
        return i

    def add_f32_wgrad(self, d):
        i = self._plan.add_f32_wgrad(d)
        self.ops.append(dict(name=d.get("name", "f32_wgrad"), reads=[d.get(k) for k in ("a1", "a2", "b")],
                             writes=[d.get("slab")]))
        return i

    def add_generic(self, kind, ptrs, ints, floats, name=""):
        i = self._plan.add_generic(kind, ptrs, ints, floats, name)
        r, w = _generic_rw(kind, list(ptrs), list(ints))
        self.ops.append(dict(name=name or kind, reads=r, writes=w,
                             spans=_generic_write_spans(kind, list(ptrs), list(ints))))
        return i

    def annotate(self, reads=(), writes=()):
        """Extra pointers of the last op (e.g. the slabs / outputs of a multi_reduce job table)."""
        self.ops[-1]["reads"] += list(reads)
        self.ops[-1]["writes"] += list(writes)

    def __getattr__(self, k):
        return getattr(self._plan, k)


class _Regions:
    def __init__(self):
        self.spans: List[Tuple[int, int, str]] = []

    def add(self, name, t):
        if isinstance(t, torch.Tensor) and t.numel() > 0:
            a = int(t.data_ptr())
            self.spans.append((a, a + t.numel() * t.element_size(), name))

    def find(self, ptr):
        s = self.find_span(ptr)
        return None if s is None else s[2]

    def find_span(self, ptr):
        best = None
        for a, b, n in self.spans:
            if a <= ptr < b and (best is None or b - a < best[1] - best[0]):
                best = (a, b, n)
        return best


def engine_regions(e) -> Tuple[_Regions, set]:
    """Named buffers of executor `e` and the subset that are step inputs."""
    R = _Regions()
    inputs = set()
    for k, t in e.bufs.items():
        R.add(k, t)
    inputs.add("x")
    for k, t in getattr(e, "relu_bits", {}).items():
        R.add("bits:" + k, t)
    for k, t in getattr(e, "pool_codes", {}).items():
        R.add("code:" + k, t)
    for k, t in getattr(e, "wcopy", {}).items():          # fp32 executor: per-step weight layouts
        R.add("wcopy:" + k, t)
    for i, t in enumerate(getattr(e, "_keep", [])):         # fp32 executor: slabs / reduction stages
        R.add("keep%d" % i, t)
    R.add("colsum_part", getattr(e, "_colsum_part", None))
    for k, t in getattr(e, "_stat_bufs", {}).items():
        R.add("stat:" + k, t)
        if k.startswith("w"):                    # bn/gn_stats workspaces (self-contained)
            inputs.add("stat:" + k)
    for k in ("prob", "target", "sums", "head_partial", "head_ws", "slab", "bias_slab", "red_stage", "arena",
              "loss_scale_dev", "_no_dy"):
        R.add(k, getattr(e, k, None))
    inputs |= {"target", "arena", "loss_scale_dev", "_no_dy"}
    for k, t in getattr(e, "state", {}).items():
        R.add("state:" + k, t)
        inputs.add("state:" + k)
    for i, t in enumerate(getattr(e, "_job_tables", [])):
        R.add("jobs%d" % i, t)
        inputs.add("jobs%d" % i)
    for tn, tf in getattr(e, "tconv_fused", {}).items():
        for k in ("wg", "hs", "bs"):
            R.add("tf:%s:%s" % (tn, k), tf[k])
        if "wa" in tf:
            R.add("tf:%s:skg" % tn, tf["wa"]["skg"])
    for k, t in getattr(e, "_dropped", {}).items():
        R.add("dropped:" + k, t)
    f = e.flat
    for name, shape, off, n in f.entries:
        R.add("master:" + name, f.view(f.master, name))
        R.add("grad:" + name, f.view(f.grad, name))
        inputs.add("master:" + name)
    return R, inputs


def check_plan(e, plan, train: bool) -> List[str]:
    """Errors of one recorded plan of executor `e` (empty list: valid)."""
    errs = []
    for i, name, err in plan.check_dispatch(0, plan.size()):
        errs.append("op %d %s: no kernel (%s)" % (i, name, err))
    R, inputs = engine_regions(e)
    written = set()
    for i, op in enumerate(plan.ops):
        for p in op["reads"]:
            if not p:
                continue
            r = R.find(int(p))
            if r is None:
                errs.append("op %d %s: reads unknown pointer 0x%x" % (i, op["name"], p))
            elif r.startswith("dropped:"):
                errs.append("op %d %s: reads %s, which the planner never forms" % (i, op["name"], r[8:]))
            elif r not in written and r not in inputs:
                errs.append("op %d %s: reads %s before any op writes it" % (i, op["name"], r))
        for p in op["writes"]:
            if not p:
                continue
            r = R.find(int(p))
            if r is None or r.startswith("dropped:") or r.startswith("master:"):
                errs.append("op %d %s: writes %s" % (i, op["name"], r or "unknown pointer 0x%x" % p))
            else:
                written.add(r)
        for p, n in op.get("spans", ()):
            sp = R.find_span(int(p))
            if sp is not None and int(p) + n > sp[1]:
                errs.append("op %d %s: writes %d bytes at %s+%d, past its end (%d bytes)"
                            % (i, op["name"], n, sp[2], int(p) - sp[0], sp[1] - sp[0]))
    if train:
        for name, shape, off, n in e.flat.entries:
            if "grad:" + name not in written:
                errs.append("no op writes the gradient of %s" % name)
    return errs


def check_engine(e) -> Dict[str, List[str]]:
    """{'train': errors, 'eval': errors} of executor `e`'s two plans."""
    return {"train": check_plan(e, e.plan, True), "eval": check_plan(e, e.eval_plan, False)}
