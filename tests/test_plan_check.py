"""Static validation of the native executor's plans across the config space (no GPU):
every fusion the planner applies meets its declarative precondition (native_engine.FUSIONS),
every planned launch resolves to a built kernel (dry dispatch), every buffer an op reads was
written earlier in the same plan (or is a step input), and every parameter gradient is
written -- for norm x decoder x dims x image size (runtime/plan_check.py)."""
import copy
import itertools

import pytest

from unet_distributed_amd.models.spec import UNetSpec
from unet_distributed_amd.parallel.grad_sync import plan_buckets
from unet_distributed_amd.runtime import native_engine as ne
from unet_distributed_amd.runtime.params import FlatParams
from unet_distributed_amd.runtime.plan_check import check_engine

CONFIGS = [(norm, ups, 2, img) for norm, ups, img in itertools.product(("none", "batch", "group"), (False, True),
                                                                      (32, 64, 128, 256))]
CONFIGS += [(norm, ups, 3, img) for norm, ups, img in itertools.product(("none", "batch"), (False, True), (16, 32))]


def _engine(norm, ups, dims, img, batch=2, opts=None, in_channels=None):
    cin = in_channels or (1 if ups else 4)
    spec = UNetSpec(in_channels=cin, use_upsampling=ups, norm=norm, dims=dims)
    flat = FlatParams(spec)
    dtype = "fp16" if norm == "group" else "bf16"
    return ne.NativeUNet(spec, flat, batch, img, "cpu", bucket_bounds=plan_buckets(flat, 4.0), dry_run=True,
                         dtype=dtype, opts=opts)


@pytest.mark.parametrize("norm,ups,dims,img", CONFIGS)
def test_every_plan_validates(norm, ups, dims, img):
    e = _engine(norm, ups, dims, img)
    errs = check_engine(e)
    assert errs == {"train": [], "eval": []}, errs
    for name, layers in e.fusions.items():
        f = ne.FUSIONS[name]
        assert not f.unmet(e), (name, f.unmet(e))
        for l in layers:
            for n in f.needs:
                assert l in e.fusions.get(n, ()), (name, l, n)


def test_headline_plan_applies_the_measured_fusions():
    e = _engine("none", False, 2, 128)
    assert sorted(e.fusions) == sorted(["head_onload", "head_fuse", "head_wsum", "pool_epilogue", "tconv_fused", "tconv_wa", "dw_fused",
                                        "tconv_onload", "skip_route", "tail_halves"])
    assert e.fusions["tconv_onload"] == ["transConv9"]


def _broken(name, **change):
    f = copy.copy(ne.FUSIONS[name])
    for k, v in change.items():
        setattr(f, k, v)
    return f


def test_validator_catches_a_broken_precondition(monkeypatch):
    """Dropping the norm restriction of the batch-half split of the last data gradient plans
    the first layer's weight gradient ahead of the norm backward that forms its operand
    coefficients: the plan builds and every kernel exists, but the weight gradient would
    read stale coefficients -- only the def-use check sees it."""
    assert check_engine(_engine("batch", False, 2, 64)) == {"train": [], "eval": []}
    monkeypatch.setitem(ne.FUSIONS, "tail_halves", _broken("tail_halves", norm=None))
    e = _engine("batch", False, 2, 64)
    errs = check_engine(e)["train"]
    assert errs and all("before any op writes it" in x for x in errs), errs
    assert any("wgrad:conv1a" in x and "ca:conv1a" in x for x in errs)


def test_tconv_onload_needs_the_chained_weight_gradient(monkeypatch):
    """A transposed conv formed on load leaves nothing to read its output: without the
    chained u-row weight gradient (tconv_wa=0) the consumer's weight gradient would read
    the never-formed u.  The declared `needs` keeps the planner from doing that; with it
    removed, planning fails loudly rather than planning a read of a dropped buffer."""
    e = _engine("none", False, 2, 64, opts=dict(tconv_wa=0))
    assert "tconv_onload" not in e.fusions and check_engine(e)["train"] == []
    monkeypatch.setitem(ne.FUSIONS, "tconv_onload", _broken("tconv_onload", needs=()))
    try:
        e = _engine("none", False, 2, 64, opts=dict(tconv_wa=0))
    except ValueError as ex:
        assert "a1" in str(ex)
    else:
        assert check_engine(e)["train"], "a read of the never-formed u went unnoticed"


def test_dry_dispatch_reports_a_missing_kernel():
    """A conv the host-side check accepts but no launcher instantiation takes is reported by
    Plan.check_dispatch (the dispatch runs on the CPU, nothing is launched)."""
    from unet_distributed_amd import native
    C = native.require()
    p = C.Plan(0)
    # dgrad-norm epilogue on a dual-source (concat) row window: accepted by
    # conv_fwd_prepare's shape checks, never instantiated (conv_win.h WIN_EPI)
    base = dict(N=1, OH=64, OW=64, IH=64, IW=64, KH=3, KW=3, pad=1, C1=32, C2=32, src1=1, src2=1, wgt=1,
                dst1=1, Cout=32, nz=1, na=1, nc=1, stats=1, npix=64 * 64, name="bad")
    try:
        p.add_conv_fwd(base)
    except ValueError:
        pytest.skip("host check rejects this combination up front")
    bad = p.check_dispatch(0, p.size())
    assert [b[1] for b in bad] == ["bad"]


@pytest.mark.parametrize("dims,img,batch,cin", [(2, 512, 128, 1), (2, 512, 64, 1), (3, 128, 16, 4), (2, 128, 2048, 4)])
def test_largest_benched_batches_plan(dims, img, batch, cin):
    """The largest per-GPU batches the config sweeps run (512^2 b128: a 2.1 GB fine gradient;
    3D b16; 2D b2048) plan without a launch refusing a > 2 GiB operand: kernels that count
    32-bit offsets from the tensor start (the transposed-conv windows) step aside for the
    per-tile-based ones there (round 5: 512^2 b128 failed after the 256-wide tconv dgrad)."""
    e = _engine("none", False, dims, img, batch=batch, in_channels=cin)
    errs = check_engine(e)
    assert errs == {"train": [], "eval": []}, errs


@pytest.mark.parametrize("dims,img,ups", [(2, 64, False), (2, 64, True), (2, 128, False), (3, 16, False),
                                          (3, 16, True)])
def test_fp32_executor_plans_validate(dims, img, ups):
    """The fp32 executor (runtime/f32_engine.py, what 'auto' picks for every fp32 GPU config)
    gets the same static dispatch / def-use / gradient-coverage validation; its dry-run
    plans refuse to run."""
    from unet_distributed_amd.runtime.f32_engine import NativeUNetF32
    spec = UNetSpec(in_channels=1 if ups else 4, use_upsampling=ups, dims=dims)
    flat = FlatParams(spec)
    e = NativeUNetF32(spec, flat, 2, img, "cpu", bucket_bounds=plan_buckets(flat, 4.0), dry_run=True)
    errs = check_engine(e)
    assert errs == {"train": [], "eval": []}, errs
    with pytest.raises(RuntimeError):
        e.forward(1)


def test_write_extent_overrun_is_flagged():
    """A write span (from the op's shape: batch chunk / channel split / slab-row offsets)
    that runs past the end of its buffer is an error, not silently accepted."""
    from unet_distributed_amd.runtime.plan_check import check_plan
    e = _engine("batch", False, 2, 64)
    assert check_plan(e, e.plan, True) == []
    k = next(i for i, op in enumerate(e.plan.ops) if op.get("spans") and op["name"].startswith("dgrad:"))
    p, n = e.plan.ops[k]["spans"][0]
    e.plan.ops[k]["spans"][0] = (p + 64, n)
    errs = check_plan(e, e.plan, True)
    assert any("past its end" in m for m in errs), errs


@pytest.mark.parametrize("norm,img", [("batch", 128), ("group", 128), ("batch", 64), ("group", 32)])
def test_dz_split_option_plans_validate(norm, img):
    """Option dz_split=1 (measured slower, off by default): the normalised layers on 16..64-wide
    rows whose dz only their own data / weight gradients read form it on load; their
    norm_bwd_apply passes and dz buffers are gone and the plan still validates (no op reads
    a dropped dz)."""
    e0 = _engine(norm, False, 2, img, batch=8)
    e1 = _engine(norm, False, 2, img, batch=8, opts=dict(dz_split=1))
    assert check_engine(e1) == {"train": [], "eval": []}
    lay = e1.fusions.get("dz_split", [])
    assert lay and not e0.fusions.get("dz_split")
    n0 = [n for n in e0.plan.names() if n.startswith("norm_bwd:")]
    n1 = [n for n in e1.plan.names() if n.startswith("norm_bwd:")]
    assert sorted(set(n0) - set(n1)) == sorted("norm_bwd:" + l for l in lay)
    assert all("dz:" + l not in e1.bufs for l in lay)


@pytest.mark.parametrize("norm,ups,img", [("none", False, 32), ("none", True, 32), ("batch", False, 32),
                                          ("none", False, 128)])
def test_route3_option_plans_validate(norm, ups, img):
    """Option route3=1: 3D decoder data gradients split, their skip half deferred to the
    pool backward's slot carrying it in the epilogue (conv_epilogue.h route_pix, 3-bit
    codes); every bwd:pool launch of the routed skips is gone and the plan validates."""
    e0 = _engine(norm, ups, 3, img, opts=dict(route3=0))
    e1 = _engine(norm, ups, 3, img, opts=dict(route3=1))
    assert check_engine(e1) == {"train": [], "eval": []}
    assert not e0.fusions.get("skip_route")
    lay = e1.fusions.get("skip_route", [])
    assert lay
    names = e1.plan.names()
    assert sum(n.startswith("dgrad_skip:") for n in names) == len(lay)
    assert sum(n.startswith("bwd:pool") for n in names) == sum(n.startswith("bwd:pool") for n in e0.plan.names()) - len(lay)


def test_head_wsum3d_option_plans_validate():
    """Option head_wsum=2 on the 3D 128^3 model: the fused-head forward accumulates the Mask
    weight sums and stores no head input; the backward forms its dY from the ReLU bits
    (head_dy) and finishes the Mask gradients from the sums; the plan validates."""
    e1 = _engine("none", False, 3, 128, batch=2, opts=dict(head_wsum=2))
    assert check_engine(e1) == {"train": [], "eval": []}
    assert e1.fusions.get("head_wsum") == ["conv9b"]
    assert "wgrad:Mask" in e1.plan.names() and "bwd:Mask" in e1.plan.names()
    e0 = _engine("none", False, 3, 128, batch=2)
    assert not e0.fusions.get("head_wsum") and "wgrad:Mask" not in e0.plan.names()


@pytest.mark.parametrize("img,batch", [(32, 2), (128, 8)])
def test_tail3_option_plans_validate(img, batch):
    """Option tail3=1: the 3D model's last data gradient runs in two volume halves with the
    first layer's weight gradient split between them; the plan validates."""
    e = _engine("none", False, 3, img, batch=batch, opts=dict(tail3=1))
    assert check_engine(e) == {"train": [], "eval": []}
    assert e.fusions.get("tail_halves") == ["conv1b"]
    assert e.plan.names().count("dgrad:conv1b") == 2 and e.plan.names().count("wgrad:conv1a") == 2
