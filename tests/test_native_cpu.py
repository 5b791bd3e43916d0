"""Native extension checks that need no GPU: the gfx950 build, the launch-plan
construction of the executor (pointers only, no launches), host-side shape
validation, bucket planning."""
import pytest
import torch

from unet_distributed_amd import native
from unet_distributed_amd.models.spec import UNetSpec
from unet_distributed_amd.parallel.grad_sync import plan_buckets
from unet_distributed_amd.runtime.params import FlatParams


def test_extension_builds_and_imports():
    native.build_if_needed()
    C = native.require()
    assert C.packseg_bytes() == 56
    assert C.crc32c(b"123456789") == 0xE3069283


@pytest.mark.parametrize("kw,img,dtype", [(dict(in_channels=4), 64, "bf16"),
                                          (dict(in_channels=1, use_upsampling=True), 64, "bf16"),
                                          (dict(in_channels=4, dims=3), 32, "bf16"), (dict(in_channels=8), 64, "bf16"),
                                          (dict(in_channels=4, norm="group"), 64, "fp16")])
def test_plan_construction_dry_run(kw, img, dtype):
    from unet_distributed_amd.runtime.native_engine import NativeUNet
    spec = UNetSpec(**kw)
    flat = FlatParams(spec)
    b = plan_buckets(flat, 4.0)
    e = NativeUNet(spec, flat, 2, img, "cpu", bucket_bounds=b, dry_run=True, dtype=dtype)
    assert e.arena.dtype == e.adt and e.target.dtype == e.adt
    names = e.plan.names()
    assert names[0] == "fwd:conv1a" and names[e.fwd_end - 1] == "fwd:Mask"
    if kw.get("dims", 2) == 2 and not kw.get("use_upsampling"):
        # default tconv_wa=1: the consumers' u-row weight gradients come from the chain rule
        # (skip-only wgrad); tconv_onload=1: nothing else reads u, so the consumers' forwards
        # form it on load -- no tconv forward launch, no fine tconv output
        assert sorted(e._wa_chain_of.values()) == ["transConv8", "transConv9"]
        for cons in e._wa_chain_of:
            assert names.index("chain:" + e._wa_chain_of[cons]) > names.index("wgrad:" + cons)
        assert sorted(e._ut_onload.values()) == ["transConv9"]          # (default: level 1)
        for t in e._ut_onload.values():
            assert "fwd:" + t not in names and t not in e.bufs
    # (head-on-load: the head backward only reduces the Mask gradients, on the side stream)
    nc = len(e.tconv_fused)
    assert [n for n in names[e.fwd_end:e.fwd_end + nc]] == ["compose:" + t for t in e.tconv_fused]
    assert names[e.fwd_end + nc] == ("wgrad:Mask" if e.head_onload else "bwd:Mask")
    # composite transposed convs (2D norm-free): no tconv data gradient, no fine output
    # gradient, the chain rule after the reduction of their slab sums
    if kw.get("dims", 2) == 2 and kw.get("norm", "none") == "none" and not kw.get("use_upsampling"):
        assert sorted(e.tconv_fused) == ["transConv8", "transConv9"]
    for t in e.tconv_fused:
        assert "dgrad:" + t not in names and "d:" + t not in e.bufs
        i = names.index("chain:" + t)
        assert any(n.startswith("reduce:") and t in n[7:].split(",") for n in names[:i])
    # every conv / tconv gradient is reduced by exactly one batched reduce op
    reduced = [ln for n in names if n.startswith("reduce:") for ln in n[len("reduce:"):].split(",")]
    assert sorted(reduced) == sorted(l.name for l in spec.param_layers() if l.kind != "mask")
    assert len(reduced) == len(set(reduced))
    # every wgrad is followed (later) by the reduce that covers its layer
    for i, n in enumerate(names):
        if n.startswith("wgrad:") and n != "wgrad:Mask":
            ln = n.split(":", 1)[1]
            assert any(m.startswith("reduce:") and ln in m[len("reduce:"):].split(",") for m in names[i + 1:])
    assert e.seg_ends[-1] == e.plan.size() and sorted(e.seg_ends) == e.seg_ends
    # dgrad of the first conv is never planned
    assert "dgrad:conv1a" not in names
    # the Adam / repack segments tile the flat buffer exactly (gaps included)
    st = e.seg_table
    assert st["off"][0] == 0 and (st["off"][1:] == st["off"][:-1] + st["n"][:-1]).all()
    assert st["off"][-1] + st["n"][-1] == flat.numel


def test_host_side_shape_validation_rejects_bad_shapes():
    C = native.require()
    base = dict(N=1, OH=8, OW=8, IH=8, IW=8, KH=3, KW=3, pad=1, src1=1, wgt=1, dst1=1, Cout=32)
    with pytest.raises(ValueError):
        C.conv_fwd(dict(base, C1=48), 0)            # Cin must be 32 / 64k
    with pytest.raises(ValueError):
        C.conv_fwd(dict(base, C1=32, Cout=40), 0)   # Cout % 32
    with pytest.raises(ValueError):
        C.wgrad(dict(N=1, QH=8, QW=8, AH=8, AW=8, KH=3, KW=3, M1=36, Nc=32, a1=1, b=1, slab=1), 0)
    with pytest.raises(ValueError):
        C.generic("pool_fwd", [1, 1], [1, 1, 8, 8, 12, 0], [], 0)


def test_tconv_onload_host_checks():
    """Transposed-conv source on load (conv_win.h XF 5): a 2D concat row-window forward,
    rows 32..128 wide, (W / 32) (C / 32) <= 8 coarse-fragment registers per row."""
    C = native.require()
    base = dict(N=1, OH=128, OW=128, IH=128, IW=128, KH=3, KW=3, pad=1, C1=32, C2=32, src1=1, src2=1, wgt=1,
                dst1=1, Cout=32, relu=1, ut_x=1, ut_w=1, ut_b=1, ut_C=64, ut_kpad=64)
    assert C.conv_fwd_grid(base) == 32
    for bad in (dict(ut_C=128, ut_kpad=128), dict(C2=0, src2=None), dict(OH=16, OW=16, IH=16, IW=16),
                dict(ut_C=48), dict(ut_kpad=32)):
        with pytest.raises(ValueError):
            C.conv_fwd_grid(dict(base, **bad))


def test_bucket_plan_is_layer_aligned_and_covers_buffer():
    spec = UNetSpec()
    flat = FlatParams(spec)
    b = plan_buckets(flat, 8.0)
    assert b[-1] == flat.numel and b == sorted(b)
    starts = {off for _, _, off, _ in flat.entries}
    for x in b[:-1]:
        assert x in starts                          # cut at a variable boundary
    # the exposed tail bucket (encoder grads, ready last) stays small
    assert (flat.numel - b[-2]) * 4 / 2 ** 20 <= 8.0


def test_engine_reads_one_env_var(monkeypatch):
    """The executor's behaviour is fixed by its measured defaults (ENGINE_DEFAULTS); the one
    environment variable it reads, UNET_ENGINE, overrides them for A/B runs, and unknown or
    removed options (the composite forward, level-3 composite backward) are errors."""
    import re
    from unet_distributed_amd.runtime import native_engine
    src = open(native_engine.__file__).read()
    assert set(re.findall(r'os\.environ\.get\("([A-Z0-9_]+)"', src)) == {"UNET_ENGINE"}
    assert "os.getenv" not in src and "os.environ[" not in src
    assert native_engine.engine_options() == native_engine.ENGINE_DEFAULTS
    monkeypatch.setenv("UNET_ENGINE", "fwd_streams=1,head_fuse=0")
    o = native_engine.engine_options(dict(dual_stream=0))
    assert (o["fwd_streams"], o["head_fuse"], o["dual_stream"], o["tconv_fused"]) == (1, 0, 0, 2)
    for bad in ("tconv_fwd=2", "tconv_fused=3"):
        monkeypatch.setenv("UNET_ENGINE", bad)
        with pytest.raises(ValueError):
            native_engine.engine_options()


def test_head_onload_plan_allocates_no_head_input_gradient():
    """Head-on-load: nothing reads or writes the head input's gradient, so it is not
    allocated (1 GiB at b1024); the materialised path keeps it."""
    from unet_distributed_amd.runtime.native_engine import NativeUNet
    spec = UNetSpec(in_channels=4)
    e = NativeUNet(spec, FlatParams(spec), 2, 64, "cpu", dry_run=True)
    assert e.head_onload and "d:" + e.head_in not in e.bufs
    e0 = NativeUNet(spec, FlatParams(spec), 2, 64, "cpu", dry_run=True, opts=dict(head_onload=0))
    assert not e0.head_onload and "d:" + e0.head_in in e0.bufs


def test_tconv_onload_plan_option():
    """tconv_onload=0 (or no chained u-row weight gradient, which reads u) keeps the
    materialised transposed-conv forward and its output tensor."""
    from unet_distributed_amd.runtime.native_engine import NativeUNet
    spec = UNetSpec(in_channels=4)
    for opts in (dict(tconv_onload=0), dict(tconv_wa=0)):
        e = NativeUNet(spec, FlatParams(spec), 2, 64, "cpu", dry_run=True, opts=opts)
        names = e.plan.names()
        assert not e._ut_onload
        for t in ("transConv8", "transConv9"):
            assert "fwd:" + t in names and t in e.bufs
    e = NativeUNet(spec, FlatParams(spec), 2, 128, "cpu", dry_run=True, opts=dict(tconv_onload=2))
    assert sorted(e._ut_onload) == ["conv8a", "conv9a"]
    # (the eval plan forms u on load too)
    assert not {"fwd:transConv8", "fwd:transConv9"} & set(e.eval_plan.names())
    e = NativeUNet(spec, FlatParams(spec), 2, 128, "cpu", dry_run=True)
    assert sorted(e._ut_onload) == ["conv9a"] and "transConv8" in e.bufs


def test_fused_head_plan():
    """The Mask head rides on the 32-channel row-window forward of its input conv
    (fwd:Mask is then only the partial reduction); norm layers or head_fuse=0 keep the
    separate head launch."""
    from unet_distributed_amd.runtime.native_engine import NativeUNet
    for kw, img, fused in [(dict(in_channels=4), 64, True), (dict(in_channels=4, dims=3), 32, True),
                           (dict(in_channels=4, norm="batch"), 64, False)]:
        spec = UNetSpec(**kw)
        e = NativeUNet(spec, FlatParams(spec), 2, img, "cpu", dry_run=True)
        assert bool(e._head_fused_blocks) == fused, kw
        assert e.plan.names()[e.fwd_end - 1] == "fwd:Mask"
    spec = UNetSpec(in_channels=4)
    e = NativeUNet(spec, FlatParams(spec), 2, 64, "cpu", dry_run=True, opts=dict(head_fuse=0))
    assert e._head_fused_blocks == 0


def test_fused_dgrad_wgrad_host_checks():
    """conv_dw.hip takes 2D 32 -> 32 channel data gradients on 128-wide rows only."""
    C = native.require()
    base = dict(N=1, OH=128, OW=128, IH=128, IW=128, KH=3, KW=3, pad=1, C1=32, src1=1, wgt=1, Cout=32, relu=0,
                dst1=1, fw_x=1, fw_slab=1, fw_bias_slab=1, fw_Cx=32, fw_nsplit=4)
    assert C.conv_fwd_grid(base) == 4
    for bad in (dict(OW=64, IW=64), dict(C1=64), dict(Cout=64, D1=64), dict(fw_nsplit=0), dict(fw_slab=None),
                dict(relu=1, bias=1)):
        with pytest.raises(ValueError):
            C.conv_fwd_grid(dict(base, **bad))


def test_persistent_window_grid():
    """win_pf > 0: the 2D 128-wide 32 -> 32 channel window runs win_pf consecutive windows
    per workgroup (grid = ceil(windows / win_pf)); any other shape keeps one window per
    workgroup, and the engine's plans carry the option on every conv launch."""
    C = native.require()
    base = dict(N=3, OH=128, OW=128, IH=128, IW=128, KH=3, KW=3, pad=1, C1=32, src1=1, wgt=1, Cout=32, relu=1,
                dst1=1)
    nwin = 3 * 128 // 4
    assert C.conv_fwd_grid(base) == nwin
    for pf in (1, 5, 8, 200):
        assert C.conv_fwd_grid(dict(base, win_pf=pf)) == (nwin + pf - 1) // pf
    for other in (dict(C1=64), dict(Cout=64), dict(OW=64, IW=64, OH=64, IH=64), dict(tile=12, Cout=64)):
        d = dict(base, **other)
        assert C.conv_fwd_grid(dict(d, win_pf=8)) == C.conv_fwd_grid(d)
