"""fp32 kernels (f32.hip, v_mfma_f32_16x16x4_f32) against fp32 ATen: the reference's own
precision (`test_dist.py:196-202`).  Products are exact in fp32 MFMA, so only the
summation order differs from ATen: relative error <= 1e-4 (observed ~1e-6)."""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, nchw, nhwc, ptr, stream

pytestmark = pytest.mark.gpu
TOL = 1e-4


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def transpose(w, T, A, B, flip):
    out = torch.empty(T * A * B, device=w.device)
    C().generic("f32_transpose", [ptr(w), ptr(out)], [T, A, B, int(flip)], [], stream())
    return out


@pytest.mark.parametrize("N,H,C1,C2,Co,relu", [(2, 16, 32, 32, 64, 1), (1, 32, 4, 0, 32, 1), (2, 8, 1, 0, 32, 0),
                                               (3, 16, 64, 0, 48, 1), (4, 128, 32, 32, 64, 1), (4, 128, 64, 0, 128, 0),
                                               (5, 128, 32, 0, 32, 1)])
def test_f32_conv3x3_fwd(cuda_dev, N, H, C1, C2, Co, relu):
    """Tiles: 128 x 32 (Cout <= 32), 128 x 64 / 128 x 128 (M >= 64k pixels), 64 x 64; the
    large shapes against the CPU (MIOpen's fp32 algorithms are no exact oracle there)."""
    torch.manual_seed(H + C1)
    dev = cuda_dev
    a = torch.randn(N, H, H, C1, device=dev)
    b = torch.randn(N, H, H, C2, device=dev) if C2 else None
    w = torch.randn(3, 3, C1 + C2, Co, device=dev) * 0.1
    bias = torch.randn(Co, device=dev)
    out = torch.empty(N, H, H, Co, device=dev)
    C().f32_conv(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(b) if C2 else None, wgt=ptr(w), bias=ptr(bias), Cout=Co, relu=relu, dst1=ptr(out)),
                 stream())
    xin = nchw(a) if not C2 else torch.cat([nchw(a), nchw(b)], 1)
    cpu = H >= 128
    dv = "cpu" if cpu else dev
    ref = nhwc(F.conv2d(xin.to(dv), w.permute(3, 2, 0, 1).to(dv), bias.to(dv), padding=1))
    if relu:
        ref = F.relu(ref)
    assert rel(out.to(dv), ref) < TOL


def test_f32_conv3d_fwd(cuda_dev):
    torch.manual_seed(3)
    dev = cuda_dev
    N, D, Ci, Co = 2, 8, 32, 32
    x = torch.randn(N, D, D, D, Ci, device=dev)
    w = torch.randn(3, 3, 3, Ci, Co, device=dev) * 0.05
    out = torch.empty(N, D, D, D, Co, device=dev)
    C().f32_conv(dict(N=N, OD=D, OH=D, OW=D, ID=D, IH=D, IW=D, KD=3, KH=3, KW=3, pad=1, C1=Ci, src1=ptr(x),
                      wgt=ptr(w), Cout=Co, relu=0, dst1=ptr(out)), stream())
    ref = F.conv3d(x.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2), padding=1).permute(0, 2, 3, 4, 1)
    assert rel(out, ref) < TOL


@pytest.mark.parametrize("C1,C2,Co", [(32, 32, 32), (32, 0, 32), (32, 0, 64), (64, 0, 64), (64, 64, 128),
                                      (4, 0, 32), (1, 0, 32)])
def test_f32_conv_dgrad_and_wgrad(cuda_dev, C1, C2, Co):
    """Data gradient = conv of dY with the flipped, transposed kernel (f32_transpose) and the
    ReLU mask of the producer; weight gradient = per-tap split-K slabs (+ the fixed-order
    slab reduction): channel-sized tiles 32 / 64 (f32_wgrad_cs_kernel, K split over the
    waves) and the generic 64 x 64 tile (channel counts not multiples of 4)."""
    torch.manual_seed(4)
    dev = cuda_dev
    N, H = 2, 32
    xa = F.relu(torch.randn(N, H, H, C1, device=dev))
    xb = F.relu(torch.randn(N, H, H, C2, device=dev))
    w = torch.randn(3, 3, C1 + C2, Co, device=dev) * 0.1
    dy = torch.randn(N, H, H, Co, device=dev)
    wd = transpose(w.reshape(-1), 9, C1 + C2, Co, True)          # [tap'][co][ci]
    dx = torch.empty(N, H, H, C1 + C2, device=dev)
    mask = torch.cat([xa, xb], -1).contiguous()
    C().f32_conv(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy), wgt=ptr(wd),
                      Cout=C1 + C2, dst1=ptr(dx), mask1=ptr(mask)), stream())
    xr = torch.cat([nchw(xa), nchw(xb)], 1).requires_grad_(True)
    wr = w.permute(3, 2, 0, 1).clone().requires_grad_(True)
    y = F.conv2d(xr, wr, padding=1)
    gx, gw = torch.autograd.grad(y, (xr, wr), nchw(dy))
    assert rel(dx, nhwc(gx) * (mask > 0)) < TOL
    splits = 5
    slab = torch.empty(splits, 9, C1 + C2, Co, device=dev)
    C().f32_wgrad(dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=C1, M2=C2, Nc=Co, a1=ptr(xa), a2=ptr(xb),
                       b=ptr(dy), slab=ptr(slab), splits=splits), stream())
    assert rel(slab.sum(0), gw.permute(2, 3, 1, 0).reshape(9, C1 + C2, Co)) < TOL


@pytest.mark.parametrize("dims", [2, 3])
def test_f32_tconv_fwd_dgrad_wgrad(cuda_dev, dims):
    torch.manual_seed(5 + dims)
    dev = cuda_dev
    N, Hc, Ci, Co = 2, 8, 64, 32
    T = 2 ** dims
    sp = (Hc,) * dims
    x = torch.randn((N,) + sp + (Ci,), device=dev)
    wt = torch.randn((2,) * dims + (Co, Ci), device=dev) * 0.1      # TF (kh, kw, Cout, Cin)
    bias = torch.randn(Co, device=dev)
    # forward: 1x1 GEMM [Ci] x [Ci][tap Co] + pixel shuffle
    wf = transpose(wt.reshape(-1), 1, T * Co, Ci, False)           # [Ci][tap][Co]
    out = torch.empty((N,) + tuple(2 * s for s in sp) + (Co,), device=dev)
    d = dict(N=N, OH=Hc, OW=Hc, IH=Hc, IW=Hc, KH=1, KW=1, C1=Ci, src1=ptr(x), wgt=ptr(wf), bias=ptr(bias),
             Cout=T * Co, shuffle=dims, dst1=ptr(out))
    if dims == 3:
        d.update(OD=Hc, ID=Hc)
    C().f32_conv(d, stream())
    perm_in = (0, 4, 1, 2, 3) if dims == 3 else (0, 3, 1, 2)
    perm_out = (0, 2, 3, 4, 1) if dims == 3 else (0, 2, 3, 1)
    wtorch = wt.permute(*((dims + 1, dims) + tuple(range(dims))))  # (Cin, Cout, k...)
    xr = x.permute(*perm_in).clone().requires_grad_(True)
    wr = wtorch.clone().requires_grad_(True)
    tfn = F.conv_transpose3d if dims == 3 else F.conv_transpose2d
    y = tfn(xr, wr, bias, stride=2)
    assert rel(out, y.permute(*perm_out)) < TOL
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (xr, wr), g)
    gf = g.permute(*perm_out).contiguous()                          # fine gradient, channels last
    # data gradient: 2x2 stride-2 conv of the fine gradient with W[tap][co][ci] (the TF layout)
    dx = torch.empty_like(x)
    d = dict(N=N, OH=Hc, OW=Hc, IH=2 * Hc, IW=2 * Hc, KH=2, KW=2, stride=2, pad=0, C1=Co, src1=ptr(gf),
             wgt=ptr(wt), Cout=Ci, dst1=ptr(dx))
    if dims == 3:
        d.update(OD=Hc, ID=2 * Hc, KD=2)
    C().f32_conv(d, stream())
    assert rel(dx, gx.permute(*perm_out)) < TOL
    # weight gradient: A = fine gradient (m = Co, taps at 2 q + tap), B = x (n = Ci)
    splits = 3
    slab = torch.empty(splits, T, Co, Ci, device=dev)
    d = dict(N=N, QH=Hc, QW=Hc, AH=2 * Hc, AW=2 * Hc, KH=2, KW=2, stride=2, pad=0, M1=Co, Nc=Ci, a1=ptr(gf),
             b=ptr(x), slab=ptr(slab), splits=splits)
    if dims == 3:
        d.update(QD=Hc, AD=2 * Hc, KD=2)
    C().f32_wgrad(d, stream())
    ref = gw.permute(*(tuple(range(2, dims + 2)) + (1, 0))).reshape(T, Co, Ci)
    assert rel(slab.sum(0), ref) < TOL


@pytest.mark.parametrize("dims", [2, 3])
def test_f32_pool_ups_head(cuda_dev, dims):
    torch.manual_seed(9 + dims)
    dev = cuda_dev
    N, S, Cc = 2, 16, 32
    D = S if dims == 3 else 1
    sp = (S,) * dims
    x = F.relu(torch.randn((N,) + sp + (Cc,), device=dev))
    y = torch.empty((N,) + tuple(s // 2 for s in sp) + (Cc,), device=dev)
    C().generic("f32_pool_fwd", [ptr(x), ptr(y)], [N, D, S, S, Cc, int(dims == 3)], [], stream())
    pool = F.max_pool3d if dims == 3 else F.max_pool2d
    perm_in = (0, 4, 1, 2, 3) if dims == 3 else (0, 3, 1, 2)
    perm_out = (0, 2, 3, 4, 1) if dims == 3 else (0, 2, 3, 1)
    xr = x.permute(*perm_in).clone().requires_grad_(True)
    yr = pool(xr, 2)
    assert torch.equal(y, yr.permute(*perm_out))
    gy = torch.randn_like(y)
    skip = torch.randn_like(x)
    dx = torch.empty_like(x)
    C().generic("f32_pool_bwd", [ptr(x), ptr(gy), ptr(skip), ptr(dx)], [N, D, S, S, Cc, int(dims == 3)], [],
                stream())
    (g,) = torch.autograd.grad(yr, xr, gy.permute(*perm_in))
    ref = (g.permute(*perm_out) + skip) * (x > 0)
    assert rel(dx, ref) < 1e-6
    # nearest upsample and its backward (sum of children, masked)
    up = torch.empty_like(x)
    C().generic("f32_ups_fwd", [ptr(y), ptr(up)], [N, max(D // 2, 1), S // 2, S // 2, Cc, int(dims == 3)], [],
                stream())
    assert torch.equal(up, F.interpolate(y.permute(*perm_in), scale_factor=2, mode="nearest").permute(*perm_out))
    dl = torch.empty_like(y)
    C().generic("f32_ups_bwd", [ptr(skip), ptr(y), ptr(dl)], [N, max(D // 2, 1), S // 2, S // 2, Cc,
                                                               int(dims == 3)], [], stream())
    k = 2
    sm = skip.permute(*perm_in)
    sm = (F.avg_pool3d(sm, k) if dims == 3 else F.avg_pool2d(sm, k)) * (k ** dims)
    assert rel(dl, sm.permute(*perm_out) * (y > 0)) < 1e-6
    # head: logits, sigmoid, Dice + BCE sums and the backward
    P = x.numel() // Cc
    w = torch.randn(Cc, device=dev) * 0.1
    b = torch.randn(1, device=dev)
    t = (torch.rand(P, device=dev) > 0.7).float()
    nb = C().f32_head_blocks(P)
    prob = torch.empty(P, device=dev)
    part = torch.empty(nb * (Cc + 1) + Cc + 1, device=dev)
    sums = torch.empty(4, device=dev)
    C().generic("f32_head_fwd", [ptr(x), ptr(w), ptr(b), ptr(t), ptr(prob), ptr(part), ptr(sums)], [P, Cc], [],
                stream())
    xf = x.reshape(P, Cc).clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    z = xf @ wr + br
    pr = torch.sigmoid(z)
    I, St, Sp = (t * pr).sum(), t.sum(), pr.sum()
    bce = F.binary_cross_entropy_with_logits(z, t, reduction="sum")
    assert rel(prob, pr) < 1e-6
    assert rel(sums, torch.stack([I, St, Sp, bce])) < 1e-5
    bce_w = 0.5
    loss = -torch.log(2 * I + 1) + torch.log(St + Sp + 1) + bce_w * bce / P
    gx, gw, gb = torch.autograd.grad(loss, (xf, wr, br))
    dxh = torch.empty_like(x)
    gwk, gbk = torch.empty(Cc, device=dev), torch.empty(1, device=dev)
    C().generic("f32_head_bwd", [ptr(x), ptr(w), ptr(prob), ptr(t), ptr(sums), ptr(dxh), ptr(part), ptr(gwk),
                                 ptr(gbk)], [P, Cc], [1.0 / P, bce_w], stream())
    assert rel(dxh.reshape(P, Cc), gx * (xf > 0)) < 1e-5
    assert rel(gwk, gw) < 1e-5 and rel(gbk, gb) < 1e-5
    # column sums (bias gradients)
    cs = torch.empty(Cc, device=dev)
    cpart = torch.empty(64 * Cc, device=dev)
    C().generic("f32_colsum", [ptr(x), ptr(cpart), ptr(cs)], [P, Cc, 64], [], stream())
    assert rel(cs, x.reshape(P, Cc).sum(0)) < 1e-6


@pytest.mark.parametrize("kw", [
    dict(batch_size=2, img_size=64, in_channels=4),
    dict(batch_size=2, img_size=64, in_channels=1, use_upsampling=True, loss="dice_bce"),
    dict(batch_size=2, img_size=16, in_channels=4, dims=3),
    dict(batch_size=3, img_size=128, in_channels=1),
])
def test_f32_native_step_matches_aten_fp32(cuda_dev, kw):
    """The whole fp32 training step (runtime/f32_engine.py: forward with dropout, Dice (+ BCE)
    loss, backward) against the fp32 ATen step on the same batch and weights, both scored
    against a float64 CPU oracle of the same step.  (MIOpen's fp32 3x3 algorithms include
    Winograd transforms, ~1e-3 relative, so the GPU ATen step is no exact-fp32 oracle; and
    two exact fp32 steps still differ where a pre-activation within rounding of zero flips a
    ReLU mask -- ~1e-4 relative on a level's weight gradient at 128^2, more than the
    summation order.)  Loss sums within 1e-5; every parameter gradient as close to float64
    as the ATen fp32 CPU step's, up to 2x + 1e-4."""
    from test_gpu_model import _setup
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.runtime.backends import TorchBackend
    from unet_distributed_amd.runtime.f32_engine import NativeUNetF32
    from unet_distributed_amd.runtime.params import FlatParams
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, dtype="fp32", backend="native", **kw)
    assert isinstance(nb.engine, NativeUNetF32)
    ft = FlatParams(spec)
    ft.master.copy_(fn.master.cpu())
    tb = TorchBackend(spec, ft, Config(**dict(kw, dtype="fp32")), "cpu", kw["batch_size"])
    nb.fwd_bwd(x, y, seed=17)
    tb.fwd_bwd(x.cpu(), y.cpu(), seed=17)
    torch.cuda.synchronize()
    assert rel(nb.sums().cpu(), tb.sums().cpu()) < 1e-5
    # float64 oracle: same leaves, batch, dropout masks (hash of seed and layer, dtype-free)
    names = [e[0] for e in ft.entries]
    leaves = {n: ft.view(ft.master, n).double().requires_grad_(True) for n in names}
    logits = reference.forward(spec, leaves, x.cpu().double(), train=True, dropout=True, seed=17, state={},
                               return_logits=True)
    t64 = y.cpu().double()
    p64 = torch.sigmoid(logits)           # (ops/losses.py total_loss, without its fp32 casts)
    loss = -torch.log(2 * (t64 * p64).sum() + 1) + torch.log(t64.sum() + p64.sum() + 1)
    if cfg.loss == "dice_bce":
        loss = loss + cfg.bce_weight * F.binary_cross_entropy_with_logits(logits, t64)
    g64 = dict(zip(names, torch.autograd.grad(loss, [leaves[n] for n in names])))
    worst = 0.0
    for name, shape, off, n in fn.entries:
        g, r = fn.grad[off:off + n].cpu(), ft.grad[off:off + n]
        o = g64[name].reshape(-1)
        e_nat, e_aten = rel(g, o), rel(r, o)
        worst = max(worst, e_nat)
        # (+5e-4: a bias gradient is a sum over every pixel with heavy cancellation, so one
        # ReLU flip near zero moves its max-norm error by up to ~1e-4 -- observed 1.3e-4 on
        # conv8a/bias at 3 x 128^2, where the CPU step happened to flip none)
        assert e_nat < 2 * e_aten + 5e-4, (name, e_nat, e_aten)
    # (flat buffers carry alignment padding between entries: compare entry by entry)
    g64_all = torch.cat([g64[name].reshape(-1) for name, _, _, _ in fn.entries])

    def l2(flat):
        a = torch.cat([flat[off:off + n].double() for _, _, off, n in fn.entries])
        return ((a - g64_all).norm() / g64_all.norm()).item()
    e_all, e_all_aten = l2(fn.grad.cpu()), l2(ft.grad)
    print("fp32 step vs float64: worst per-tensor %.2e, all gradients L2 %.2e (ATen fp32 CPU %.2e)"
          % (worst, e_all, e_all_aten))
    assert e_all < 2 * e_all_aten + 1e-5
    # the fused TF-Adam launch on the fp32 master (no 16-bit repack) against the torch
    # TF-Adam on the same gradient (Adam's first step is ~lr sign(g): gradients within
    # rounding of zero would flip it, so both updates see the native gradient)
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.trainer import _NativeOpt
    ft.grad.copy_(fn.grad.cpu())
    opt_n, opt_t = TFAdam(fn, cfg, native=_NativeOpt(nb)), TFAdam(ft, cfg)
    opt_n.step()
    opt_t.step()
    torch.cuda.synchronize()
    assert rel(fn.master.cpu(), ft.master) < 1e-6
