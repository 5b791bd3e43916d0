"""Whole-step parity: the native HIP executor (bf16 MFMA kernels) against the
fp32 ATen reference of the same UNet, same weights, same batch, same dropout
masks (shared counter hash)."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda_dev, **kw):
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.runtime.backends import NativeBackend, TorchBackend
    from unet_distributed_amd.runtime.params import FlatParams
    cfg = Config(**kw)
    spec = spec_from_config(cfg)
    B = cfg.batch_size
    x, y = synthetic_brats(B, cfg.img_size, cfg.in_channels, cfg.dims, seed=5)
    x, y = torch.from_numpy(x).to(cuda_dev), torch.from_numpy(y).to(cuda_dev)
    init = reference.init_params(spec, seed=3)
    fn = FlatParams(spec, device=cuda_dev)
    fn.load_dict(init)
    nb = NativeBackend(spec, fn, cfg, cuda_dev, B)
    cfg32 = Config(**dict(kw, dtype="fp32"))
    ft = FlatParams(spec, device=cuda_dev)
    ft.load_dict(init)
    tb = TorchBackend(spec, ft, cfg32, cuda_dev, B)
    return spec, cfg, x, y, fn, nb, ft, tb


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _grad_parity(fn, ft, tag):
    """Per-variable (1 - cosine, |norm ratio - 1|) of the native gradients against the fp32
    ATen step; logged (and written to gpurun_out/parity.jsonl on the GPU box) so the bounds
    below track the observed worst case (about 2x of it)."""
    import json
    rows = {}
    for name, shape, off, n in fn.entries:
        gn, gt = fn.grad[off:off + n], ft.grad[off:off + n]
        if gt.norm() < 1e-6:          # conv bias under BatchNorm: exactly 0 in exact arithmetic
            assert gn.norm() < 1e-3, (name, gn.norm().item())
            continue
        rows[name] = (1.0 - _cos(gn, gt), abs((gn.norm() / (gt.norm() + 1e-30)).item() - 1.0))
    worst_k = max((v[0], k) for k, v in rows.items() if not k.endswith("/bias"))
    worst_b = max(((v[0], k) for k, v in rows.items() if k.endswith("/bias")), default=(0.0, None))
    worst_r = max((v[1], k) for k, v in rows.items())
    rec = dict(tag=tag, worst_cos_dist_kernel=worst_k, worst_cos_dist_bias=worst_b, worst_ratio_dev=worst_r,
               total_cos_dist=1.0 - _cos(fn.grad, ft.grad))
    print("parity", json.dumps(rec))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "parity.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    return rows, rec


# Whole-step parity bounds (1 - cosine of a kernel / bias gradient, |norm ratio - 1|, 1 - cosine
# of the whole gradient) at about 2x the worst values observed on the GPU (round 4,
# gpurun_out/parity.jsonl: e.g. the shipped shape at batch 64 -- 0.0029 / 0.0029 / 0.021 /
# 1.4e-5), capped by the round-3 bounds (0.02 / 0.05 / 0.1 / 0.01).  The small-batch configs
# (2-4 images) sum bf16 rounding over few pixels and sit close to the caps; the shipped
# shape is held an order of magnitude tighter, where a 5 % scale error in one layer fails.
PARITY_BOUNDS = {
    "shipped:B=64": (0.006, 0.006, 0.045, 1e-4),
    "shipped:B=256": (0.006, 0.006, 0.045, 1e-4),
    "step:batch_size=2,img_size=256,in_channels=1": (0.02, 0.03, 0.045, 1e-4),
    "step:batch_size=2,dims=3,img_size=32,in_channels=4": (0.02, 0.03, 0.045, 5e-4),
    "step:batch_size=4,img_size=64,in_channels=4": (0.02, 0.037, 0.1, 3e-4),
    "step:batch_size=4,img_size=64,in_channels=4,loss=dice_bce": (0.02, 0.037, 0.062, 4e-4),
    # the 1-channel upsampling step at batch 2 sits at ATen's own bf16 noise floor: total
    # distance native 0.0062 vs ATen bf16 autocast 0.0057 on the same step, 0.0021 / 0.0018
    # at batch 8, native fp32 1e-12 (scripts/ups_parity_diag.py, profiles/r5_ups_parity_diag.md)
    "step:batch_size=2,img_size=64,in_channels=1,use_upsampling=True": (0.02, 0.037, 0.1, 0.01),
}


def _check_parity(rows, rec):
    kb, bb, rb, tb = PARITY_BOUNDS.get(rec["tag"], (0.02, 0.05, 0.1, 0.01))
    for name, (dc, dr) in rows.items():
        assert dc < (bb if name.endswith("/bias") else kb), (rec["tag"], name, dc)
        assert dr < rb, (rec["tag"], name, dr)
    assert rec["total_cos_dist"] < tb, rec


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=64, in_channels=4),
    dict(batch_size=2, img_size=64, in_channels=1, use_upsampling=True),
    dict(batch_size=4, img_size=64, in_channels=4, loss="dice_bce"),
    dict(batch_size=2, img_size=32, in_channels=4, dims=3),
    dict(batch_size=2, img_size=256, in_channels=1),
])
def test_native_step_matches_reference(cuda_dev, kw):
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
    nb.fwd_bwd(x, y, seed=77)
    tb.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    sn, st = nb.sums().cpu(), tb.sums().cpu()
    assert torch.allclose(sn[:3], st[:3], rtol=3e-2, atol=1.0), (sn, st)
    _check_parity(*_grad_parity(fn, ft, "step:" + ",".join("%s=%s" % kv for kv in sorted(kw.items()))))


@pytest.mark.parametrize("B", [64, 256])
def test_native_step_matches_reference_at_shipped_shape(cuda_dev, B):
    """The benchmarked configuration itself: 128x128x4, bf16, per-GPU batch 64 and 256 (the
    reference's per-worker batch) with the production split-K sizing (wg_target),
    dual-stream backward, HIP-graph forward and the fused segmentation head; gradients vs
    the fp32 ATen step.  (At the bench's 1024 the fp32 ATen reference step -- MIOpen
    searching fp32 algorithms for new shapes -- outlasted the GPU runner's silence limit.)"""
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=B, img_size=128, in_channels=4,
                                              hip_graph=True)
    e = nb.engine
    assert e.dual_stream and e._head_fused_blocks > 0 and e.graphs is not None
    for rep in range(2):                       # second pass replays the captured graphs
        nb.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    print("native step done", flush=True)
    tb.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    print("ATen fp32 step done", flush=True)
    sn, st = nb.sums().cpu(), tb.sums().cpu()
    assert torch.allclose(sn[:3], st[:3], rtol=2e-2, atol=1.0), (sn, st)
    _check_parity(*_grad_parity(fn, ft, "shipped:B=%d" % B))


def test_native_adam_matches_reference(cuda_dev):
    from unet_distributed_amd.runtime.optim import adam_reference_
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=2, img_size=32, in_channels=4)
    g = torch.randn(fn.numel, device=cuda_dev) * 1e-2
    fn.grad.copy_(g)
    w0 = fn.master.clone()
    nb.adam_step(5e-4, 0.9, 0.999)
    w, m, v = w0.clone(), torch.zeros_like(w0), torch.zeros_like(w0)
    adam_reference_(w, g, m, v, 5e-4, 0.9, 0.999)
    torch.cuda.synchronize()
    assert torch.allclose(fn.master, w, rtol=1e-5, atol=1e-7)
    assert torch.allclose(fn.m, m) and torch.allclose(fn.v, v)
    # the 16-bit compute copies written by the Adam launch equal a plain repack of the
    # updated master (every kernel layout, both copies, padding untouched)
    a1 = nb.engine.arena.clone()
    nb.engine.repack()
    torch.cuda.synchronize()
    assert torch.equal(a1, nb.engine.arena)
    assert (a1 != 0).sum().item() >= spec.num_params() - 1000


def test_native_training_reduces_loss(cuda_dev):
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.trainer import _NativeOpt
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=8, img_size=64, in_channels=4,
                                              learning_rate=1e-3)
    opt = TFAdam(fn, cfg, native=_NativeOpt(nb))
    losses = []
    for i in range(30):
        nb.fwd_bwd(x, y, seed=i)
        opt.step()
        s = nb.sums().cpu()
        losses.append((-torch.log(2 * s[0] + 1) + torch.log(s[1] + s[2] + 1)).item())
    assert losses[-1] < 0.7 * losses[0], losses


def test_native_inference_export_roundtrip(cuda_dev, tmp_path):
    """export -> load_saved_model on the GPU runs the native eval plan; probabilities
    match the fp32 reference forward (dropout off), short tail batch padded."""
    import numpy as np
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.inference import load_saved_model
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.utils.checkpoint import export_model
    cfg = Config(img_size=64, in_channels=4, checkpoint_dir=str(tmp_path))
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=3))
    d = export_model(cfg, spec, flat)
    os.remove(os.path.join(d, "saved_model.json"))          # the GraphDef alone describes the model
    model = load_saved_model(d, device=cuda_dev, batch=4)
    assert model.name == "native"
    x, _ = synthetic_brats(6, 64, 4, seed=2)
    p = model.predict(x)
    with torch.no_grad():
        ref = reference.forward(spec, {k: v.to(cuda_dev) for k, v in flat.params().items()},
                                torch.from_numpy(x).to(cuda_dev), train=False, dropout=False).cpu().numpy()
    assert p.shape == ref.shape
    assert np.abs(p - ref).max() < 0.05, np.abs(p - ref).max()


@pytest.mark.parametrize("norm", ["batch", "group"])
def test_native_norm_state_and_eval(cuda_dev, norm):
    """BatchNorm running statistics follow the ATen momentum update; eval-mode sums
    (BN: running stats, GN: per-sample stats) match the fp32 reference."""
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=4, img_size=64, in_channels=4, norm=norm)
    for k in range(2):
        nb.fwd_bwd(x, y, seed=5 + k)
        tb.fwd_bwd(x, y, seed=5 + k)
    torch.cuda.synchronize()
    if norm == "batch":
        assert set(nb.state) == set(tb.state)
        for k in tb.state:
            a, b = nb.state[k].float(), tb.state[k].float()
            assert torch.allclose(a, b, rtol=3e-2, atol=3e-2), (k, (a - b).abs().max().item())
    en, et = nb.eval_sums(x, y).cpu(), tb.eval_sums(x, y).cpu()
    assert torch.allclose(en[:3], et[:3], rtol=5e-2, atol=2.0), (en, et)


@pytest.mark.parametrize("norm", ["batch", "group"])
def test_native_norm_step_matches_bf16_noise_floor(cuda_dev, norm):
    """With BatchNorm / GroupNorm the backward cancels large terms, so any bf16 storage
    drifts from fp32 layer by layer (ATen's own bf16 autocast reaches cos ~0.93 at the
    bottleneck).  The native step must track the fp32 gradients at least as well as
    ATen bf16 does (per layer, within 0.02) and match fp32 overall."""
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.runtime.backends import TorchBackend
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.models import reference
    kw = dict(batch_size=4, img_size=64, in_channels=4, norm=norm, groups=8)
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
    fb = FlatParams(spec, device=cuda_dev)
    fb.load_dict(reference.init_params(spec, seed=3))
    bb = TorchBackend(spec, fb, Config(**dict(kw, dtype="bf16")), cuda_dev, 4)
    for be in (nb, tb, bb):
        be.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    cns, cbs = [], []
    for name, shape, off, n in fn.entries:
        g32 = ft.grad[off:off + n]
        if g32.norm() < 1e-6:
            continue
        cn, cb = _cos(fn.grad[off:off + n], g32), _cos(fb.grad[off:off + n], g32)
        # single layers at the bottleneck scatter by ~+-0.02 around the floor
        assert cn > cb - 0.04, (name, cn, cb)
        cns.append(cn)
        cbs.append(cb)
    assert sum(cns) / len(cns) > sum(cbs) / len(cbs) - 0.005, (cns, cbs)
    assert _cos(fn.grad, ft.grad) > 0.98


@pytest.mark.parametrize("norm", ["none", "batch"])
def test_hip_graph_replay_equals_eager(cuda_dev, monkeypatch, norm):
    """Graph mode (captured fwd, per-bucket bwd segments, Adam reading its scalars from
    device memory) is bit-identical to eager plan replay over several steps with
    changing dropout seeds and learning rates.  (One-stream forward: the two-stream
    forward is launched eagerly even in graph mode.)"""
    monkeypatch.setenv("UNET_ENGINE", "fwd_streams=1")
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.parallel.grad_sync import plan_buckets
    from unet_distributed_amd.runtime.backends import NativeBackend
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.runtime.trainer import _NativeOpt
    runs = []
    for graph in (False, True):
        cfg = Config(batch_size=4, img_size=64, in_channels=4, norm=norm, hip_graph=graph,
                     learning_rate=1e-3)
        spec = spec_from_config(cfg)
        x, y = synthetic_brats(4, 64, 4, 2, seed=5)
        x, y = torch.from_numpy(x).to(cuda_dev), torch.from_numpy(y).to(cuda_dev)
        fl = FlatParams(spec, device=cuda_dev)
        fl.load_dict(reference.init_params(spec, seed=3))
        bounds = plan_buckets(fl, 1.0)
        nb = NativeBackend(spec, fl, cfg, cuda_dev, 4, bounds)
        nb.engine.repack()
        assert (nb.engine.graphs is not None) == graph
        opt = TFAdam(fl, cfg, native=_NativeOpt(nb))
        seen = []
        for i in range(3):
            nb.fwd_bwd(x, y, seed=1000 + 7 * i, on_segment=seen.append)
            opt.step()
        torch.cuda.synchronize()
        assert seen == list(range(len(nb.engine.seg_ends))) * 3
        runs.append((fl.master.clone(), fl.m.clone(), nb.sums().clone()))
        if graph:
            # the captured forward really holds the kernels (not launched eagerly at capture)
            e = nb.engine
            e.sums.zero_()
            e.graphs[("fwd", e.fwd_end)].replay()
            torch.cuda.synchronize()
            assert e.sums[1].item() > 0
    (w0, m0, s0), (w1, m1, s1) = runs
    assert torch.equal(s0, s1)
    assert torch.equal(m0, m1)
    assert torch.equal(w0, w1)


@pytest.mark.parametrize("kw", [
    dict(batch_size=8, img_size=64, in_channels=4, dropout=0.0),
    dict(batch_size=4, img_size=64, in_channels=1, use_upsampling=True, hip_graph=True, dropout=0.0),
    dict(batch_size=4, img_size=64, in_channels=4),
    dict(batch_size=4, img_size=64, in_channels=4, norm="group", dtype="fp16"),
    dict(batch_size=6, img_size=128, in_channels=4, norm="group", dtype="fp16", loss="dice_bce"),
    dict(batch_size=4, img_size=64, in_channels=1, use_upsampling=True, norm="group"),
])
def test_two_stream_forward_equals_one_stream(cuda_dev, monkeypatch, kw):
    """fwd_streams=2 runs the training forward as two half-batch chunks on two
    streams (fused pools / head logits written at the chunk's offset): activations,
    loss sums and gradients are bit-identical to the one-stream forward, dropout
    included (each chunk hashes its elements' whole-batch indices, drop_idx0 / the
    norm pass's n0).  GroupNorm: each chunk finalizes its own samples' statistics at
    its offset, the head input's normalisation + loss sums run on the whole batch."""
    outs = []
    for n in ("1", "2"):
        monkeypatch.setenv("UNET_ENGINE", "fwd_streams=" + n)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        assert (getattr(nb.engine, "_fwd2", None) is not None) == (n == "2")
        for seed in (77, 0x9E3779B9):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), nb.engine.prob.clone(), fn.grad.clone(),
                     nb.engine.bufs["conv5b"].clone()))
    (s0, p0, g0, a0), (s1, p1, g1, a1) = outs
    assert torch.equal(a0, a1)
    assert torch.equal(p0, p1)
    assert torch.equal(s0, s1)
    assert torch.equal(g0, g1)


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=64, in_channels=4, loss="dice_bce"),
    dict(batch_size=2, img_size=32, in_channels=4, dims=3),
])
def test_fused_head_matches_separate_head(cuda_dev, monkeypatch, kw):
    """The head fused into the head-input conv's epilogue (head_fuse=1) gives the
    separate head kernel's probabilities, loss sums and gradients up to fp32
    summation order."""
    outs = []
    for f in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "head_fuse=" + f)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        assert bool(nb.engine._head_fused_blocks) == (f == "1")
        nb.fwd_bwd(x, y, seed=77)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), nb.engine.prob.clone(), fn.grad.clone()))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-2), (s0, s1)
    assert (p0 - p1).abs().max().item() < 1e-5
    assert _cos(g0, g1) > 0.99999


@pytest.mark.parametrize("norm", ["batch", "group"])
def test_native_inference_export_roundtrip_norm(cuda_dev, tmp_path, norm):
    """A --norm batch|group export served by the native eval plan: the BatchNorm
    moving statistics written with the export are the ones the native plan
    normalises with (non-trivial stats, so mean 0 / var 1 would fail)."""
    import numpy as np
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.inference import load_saved_model
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.utils.checkpoint import export_model
    cfg = Config(img_size=64, in_channels=4, checkpoint_dir=str(tmp_path), norm=norm)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=3))
    g = torch.Generator().manual_seed(0)
    state = {}
    if norm == "batch":
        for l in spec.param_layers():
            if l.kind == "conv":
                state[l.name + "/norm/moving_mean"] = 0.2 * torch.randn(l.cout, generator=g)
                state[l.name + "/norm/moving_variance"] = 0.5 + torch.rand(l.cout, generator=g)
    d = export_model(cfg, spec, flat, extra_state=state)
    os.remove(os.path.join(d, "saved_model.json"))
    model = load_saved_model(d, device=cuda_dev, batch=4)
    assert model.name == "native"
    x, _ = synthetic_brats(4, 64, 4, seed=2)
    p = model.predict(x)
    with torch.no_grad():
        ref = reference.forward(spec, {k: v.to(cuda_dev) for k, v in flat.params().items()},
                                torch.from_numpy(x).to(cuda_dev), train=False, dropout=False,
                                state={k: v.to(cuda_dev) for k, v in state.items()}).cpu().numpy()
    assert np.abs(p - ref).max() < 0.05, np.abs(p - ref).max()


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=64, in_channels=4),
    dict(batch_size=4, img_size=128, in_channels=4, loss="dice_bce", hip_graph=True),
    dict(batch_size=2, img_size=32, in_channels=4, dims=3),
    dict(batch_size=1, img_size=64, in_channels=4, dims=3, loss="dice_bce"),
])
def test_head_onload_step_equals_materialised(cuda_dev, monkeypatch, kw):
    """head_onload=1 (default: the head input's gradient formed on load by its
    consumers, no dY tensor) gives the materialised-dY step bit for bit: loss sums,
    probabilities and every parameter gradient."""
    outs = []
    for v in ("0", "2"):
        # (head_onload=2: 3D too; dw_fuse=0: with head_onload=0 the head input conv's weight gradient would run in
        # the fused data + weight gradient kernel, a different fp32 summation order)
        # (head_wsum=0: the Mask gradients from head_bwd on both sides -- the forward sums
        # of head_wsum round differently, test_head_wsum_step_matches below)
        monkeypatch.setenv("UNET_ENGINE", "dw_fuse=0,head_wsum=0,head_onload=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert e.head_onload == (v == "2")
        assert ("wgrad:Mask" in e.plan.names()) == (v == "2")
        for seed in (77, 78):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), fn.grad.clone()))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    assert torch.equal(g0, g1)


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=128, in_channels=4),
    dict(batch_size=6, img_size=128, in_channels=4, loss="dice_bce", hip_graph=True),
    dict(batch_size=2, img_size=128, in_channels=4, dtype="fp16"),
])
def test_head_wsum_step_matches(cuda_dev, monkeypatch, kw):
    """head_wsum=1 (default: the Mask gradients from per-workgroup sums of the fused-head
    forward, the head input never stored) vs head_wsum=0 (head_bwd re-reads the stored head
    input): identical loss sums, probabilities and every other gradient bit for bit; the
    Mask weight / bias gradients equal up to fp32 summation order."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "head_wsum=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert bool(e.fusions.get("head_wsum")) == (v == "1")
        for seed in (61, 62):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        if k.startswith("Mask/"):
            err = ((g1[k] - g0[k]).abs().max() / (g0[k].abs().max() + 1e-12)).item()
            assert err < 1e-4, (k, err)
        else:
            assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=64, in_channels=4),
    dict(batch_size=4, img_size=128, in_channels=4, loss="dice_bce"),
])
def test_tconv_fused_step_matches_materialised(cuda_dev, monkeypatch, kw):
    """Composite transposed-conv backward (default, levels 1-2: no fine tconv output
    gradient) vs tconv_fused=0 (dgrad into d:transConv, tconv dgrad / wgrad):
    same loss sums and probabilities, every parameter gradient within bf16 rounding of
    the other path (the composed weights round once instead of twice)."""
    outs = []
    for v in ("0", "2"):
        # (tconv_wa=0: the consumer's full weight gradient; the chained one: next test)
        monkeypatch.setenv("UNET_ENGINE", "tconv_wa=0,tconv_fused=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert sorted(e.tconv_fused) == ([] if v == "0" else ["transConv8", "transConv9"])
        nb.fwd_bwd(x, y, seed=91)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)      # the forward is unchanged
    for k in g0:
        a, b = g1[k].float(), g0[k].float()
        err = ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()
        assert err < 3e-2 and _cos(a, b) > 0.999, (k, err, _cos(a, b))


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=64, in_channels=4),
    dict(batch_size=4, img_size=128, in_channels=4, loss="dice_bce"),
])
def test_tconv_consumer_modes_step(cuda_dev, monkeypatch, kw):
    """tconv_wa 0 (tconv + fine conv, full wgrad) and 1 (default: the consumer's u-row
    weight gradient from the slab sums, skip-only wgrad).  The forward is bit-identical; mode 1
    rounds differently from mode 0 (u is never rounded to 16 bits on its u-row gradient path),
    so both are held against the fp32 ATen step and mode 1 must be as close to it as mode 0
    (per-gradient cosine distance at most 2x + 3e-4 of mode 0's)."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "tconv_wa=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert sorted(e._wa_chain_of.values()) == ([] if v == "0" else ["transConv8", "transConv9"])
        nb.fwd_bwd(x, y, seed=91)
        if v == "0":
            tb.fwd_bwd(x, y, seed=91)
            ref = (tb.sums().cpu(), {k: ft.view(ft.grad, k).clone() for k, *_ in ft.entries})
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    st, gt = ref
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        d0 = 1.0 - _cos(g0[k].float(), gt[k])
        d = 1.0 - _cos(g1[k].float(), gt[k])
        assert d <= 2.0 * d0 + 3e-4, (k, d0, d)


@pytest.mark.parametrize("norm", ["batch", "group"])
def test_tconv_fused_norm_step(cuda_dev, monkeypatch, norm):
    """Composite transposed-conv backward with BatchNorm / GroupNorm (the S2D data gradient
    carries the tconv input's dgrad-norm epilogue; the consumer's u-row weight gradient
    from the slab sums) vs the materialised tconv backward (tconv_fused=0): both held
    against the fp32 ATen step, the composite at most 2x + 1e-3 the materialised path's
    per-gradient cosine distance."""
    outs = []
    for v in ("0", "2"):
        monkeypatch.setenv("UNET_ENGINE", "tconv_fused=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=4, img_size=64, in_channels=4, norm=norm)
        e = nb.engine
        assert sorted(e.tconv_fused) == ([] if v == "0" else ["transConv8", "transConv9"])
        nb.fwd_bwd(x, y, seed=93)
        if v == "0":
            tb.fwd_bwd(x, y, seed=93)
            ref = {k: ft.view(ft.grad, k).clone() for k, *_ in ft.entries}
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, g0), (s2, g2) = outs
    assert torch.equal(s0, s2)                               # the forward is unchanged
    for k in g0:
        if ref[k].norm() < 1e-6:
            continue
        d0 = 1.0 - _cos(g0[k].float(), ref[k])
        d2 = 1.0 - _cos(g2[k].float(), ref[k])
        assert d2 <= 2.0 * d0 + 1e-3, (k, d0, d2)


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=128, in_channels=4),
    dict(batch_size=3, img_size=128, in_channels=4, loss="dice_bce", hip_graph=True),
])
def test_fused_dgrad_wgrad_step(cuda_dev, monkeypatch, kw):
    """dw_fuse=1 (default: conv1b's and conv9b's data and weight gradients from one staged
    dY halo -- conv9b's formed on load from the head, conv_dw.hip XF 4) vs dw_fuse=0: the forward, every data gradient and every other parameter
    gradient are bit-identical; the fused layers' weight / bias gradients differ only by
    fp32 summation order."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "dw_fuse=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        fused = sorted(e.fusions.get("dw_fused", []))
        assert (fused == ["conv1b", "conv9b"]) == (v == "1"), fused
        for seed in (31, 32):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), e.bufs["d:conv1a"].clone(),
                     {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, d0, g0), (s1, p1, d1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1) and torch.equal(d0, d1)
    for k in g0:
        if k.startswith(("conv1b/", "conv9b/")):
            assert rel_err_(g1[k], g0[k]) < 1e-5, (k, rel_err_(g1[k], g0[k]))
        else:
            assert torch.equal(g0[k], g1[k]), k


def rel_err_(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


@pytest.mark.parametrize("norm,dtype", [("batch", "bf16"), ("group", "fp16")])
def test_fused_dgrad_wgrad_norm_step(cuda_dev, monkeypatch, norm, dtype):
    """Normalised configs at 128^2: dw_fuse=1 runs conv1b / conv9b's data + weight gradients
    in one kernel with their norm backward's dz formed on load (conv_dw XF 2 / XF 3: no
    norm_bwd_apply / head_norm_bwd pass) vs dw_fuse=0 (split kernels, materialised dz).
    The forward is bit-identical; the backward differs only by the statistics rows'
    summation order (per 256-pixel window instead of per split-kernel tile)."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "dw_fuse=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=4, img_size=128, in_channels=4, norm=norm,
                                                 groups=8, dtype=dtype)
        e = nb.engine
        assert sorted(e.fusions.get("dz_onload", [])) == (["conv1b", "conv9b"] if v == "1" else []), e.fusions
        names = e.plan.names()
        assert ("norm_bwd:conv1b" in names) == (v == "0") and ("norm_bwd:conv9b" in names) == (v == "0")
        nb.fwd_bwd(x, y, seed=41)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        if norm == "batch" and k.endswith("/bias") and not k.startswith("Mask"):
            continue       # (a conv bias before BatchNorm: analytically zero gradient, rounding noise)
        if g0[k].norm() > 1e-6:
            assert _cos(g1[k], g0[k]) > 0.999, (k, _cos(g1[k], g0[k]))


@pytest.mark.parametrize("kw", [
    dict(batch_size=4, img_size=128, in_channels=4, norm="batch"),
    dict(batch_size=3, img_size=128, in_channels=4, norm="batch", loss="dice_bce", hip_graph=True),
    dict(batch_size=4, img_size=128, in_channels=4, norm="group", dtype="fp16"),
    dict(batch_size=6, img_size=128, in_channels=4, norm="group", hip_graph=True),
])
def test_skip_onload_step_equals_materialised(cuda_dev, monkeypatch, kw):
    """skip_onload=1 (normalised configs' default: conv9a's skip source conv1b is never stored in
    training -- the tconv-on-load forward and the chained skip-row weight gradient normalise
    its pre-norm z on load with norm_pool's formula) gives the materialised step bit for bit:
    loss sums, probabilities, every parameter gradient."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "skip_onload=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert bool(e.fusions.get("skip_onload")) == (v == "1")
        for seed in (41, 42):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), fn.grad.clone()))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    assert torch.equal(g0, g1)


@pytest.mark.parametrize("kw", [
    dict(batch_size=2, img_size=32, in_channels=4, dims=3),
    dict(batch_size=1, img_size=64, in_channels=4, dims=3, loss="dice_bce"),
    dict(batch_size=2, img_size=32, in_channels=4, dims=3, norm="batch"),
])
def test_route3_step_equals_separate_pool_bwd(cuda_dev, monkeypatch, kw):
    """3D skip_route (route3=1: the decoder data gradients split, the skip half deferred and
    carrying the pool backward in its epilogue with 3-bit window codes) vs the dual-destination
    data gradient + separate pool backward: loss sums and probabilities bit for bit, parameter
    gradients to rounding (the split halves' MFMA tiles may differ)."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "route3=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert bool(e.fusions.get("skip_route")) == (v == "1")
        nb.fwd_bwd(x, y, seed=41)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        if kw.get("norm") == "batch" and k.endswith("/bias") and not k.startswith("Mask"):
            continue
        if g0[k].norm() > 1e-6:
            assert rel_err_(g1[k], g0[k]) < 2e-3, (k, rel_err_(g1[k], g0[k]))


@pytest.mark.parametrize("kw", [
    dict(batch_size=1, img_size=128, in_channels=4, dims=3),
    dict(batch_size=2, img_size=128, in_channels=4, dims=3, loss="dice_bce"),
])
def test_head_wsum3d_step_matches(cuda_dev, monkeypatch, kw):
    """3D head_wsum=2 (the 128-wide chunk-pipelined fused-head forward accumulates the Mask
    weight sums and does not store the head input; head_dy forms the head input's dY from its
    ReLU bits) vs head_wsum=1 (3D: head_bwd re-reads the stored head input): identical loss
    sums, probabilities and every other gradient bit for bit; the Mask gradients equal up to
    fp32 summation order."""
    outs = []
    for v in ("1", "2"):
        monkeypatch.setenv("UNET_ENGINE", "head_wsum=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert bool(e.fusions.get("head_wsum")) == (v == "2")
        assert ("wgrad:Mask" in e.plan.names()) == (v == "2")
        for seed in (61, 62):
            nb.fwd_bwd(x, y, seed=seed)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        if k.startswith("Mask/"):
            err = ((g1[k] - g0[k]).abs().max() / (g0[k].abs().max() + 1e-12)).item()
            assert err < 1e-4, (k, err)
        else:
            assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("kw", [
    dict(batch_size=2, img_size=32, in_channels=4, dims=3),
    dict(batch_size=2, img_size=128, in_channels=4, dims=3, loss="dice_bce"),
])
def test_tail3_step_matches(cuda_dev, monkeypatch, kw):
    """3D tail halves (tail3=1: the last data gradient in two batch halves, the first layer's
    weight gradient split at the same volume boundary so its first half overlaps the second
    data-gradient half) vs one launch each: loss sums and probabilities bit for bit, gradients to
    split-K summation order."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("UNET_ENGINE", "tail3=" + v)
        spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, **kw)
        e = nb.engine
        assert bool(e.fusions.get("tail_halves")) == (v == "1")
        nb.fwd_bwd(x, y, seed=41)
        torch.cuda.synchronize()
        outs.append((nb.sums().cpu(), e.prob.clone(), {k: fn.view(fn.grad, k).clone() for k, *_ in fn.entries}))
    (s0, p0, g0), (s1, p1, g1) = outs
    assert torch.equal(s0, s1) and torch.equal(p0, p1)
    for k in g0:
        if g0[k].norm() > 1e-6:
            assert rel_err_(g1[k], g0[k]) < 1e-3, (k, rel_err_(g1[k], g0[k]))
