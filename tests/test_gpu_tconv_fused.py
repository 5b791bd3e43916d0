"""Composite transposed-conv backward (tconv_fused.hip + conv_win.h XF 4) against an
fp32 autograd reference of the decoder step u = tconv(b); z = conv3x3([u, skip]).

The data gradient of b is one coarse 3x3 row-window conv over the space-to-depth image
of dz with composed weights; the tconv weight / bias gradients come from the 4x4-tap
stride-2 slab sums through the chain rule.  du is never formed."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def C():
    from unet_distributed_amd import native
    return native.require()


def ptr(t):
    return int(t.data_ptr())


def stream():
    return int(torch.cuda.current_stream().cuda_stream)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def nchw(x):
    return x.permute(0, 3, 1, 2)


def nhwc(x):
    return x.permute(0, 2, 3, 1)


def pack_bits(y):
    pos = (y.float() > 0).to(torch.int32).reshape(*y.shape[:-1], y.shape[-1] // 8, 8)
    return (pos << torch.arange(8, device=y.device, dtype=torch.int32)).sum(-1).to(torch.uint8)


def _problem(dev, N, H, K, Cc, Cs, O, seed):
    torch.manual_seed(seed)
    b = F.relu(torch.randn(N, H, H, K, device=dev)).bfloat16()
    skip = torch.randn(N, 2 * H, 2 * H, Cs, device=dev).bfloat16()
    wt = torch.randn(2, 2, Cc, K, device=dev) * 0.1          # Keras Conv2DTranspose (kh, kw, Cout, Cin)
    bt = torch.randn(Cc, device=dev) * 0.1
    wa = torch.randn(3, 3, Cc + Cs, O, device=dev) * 0.1      # HWIO, u channels first
    dz = torch.randn(N, 2 * H, 2 * H, O, device=dev).bfloat16()
    return b, skip, wt, bt, wa, dz


def _reference(b, skip, wt, bt, wa, dz, with_wa=False):
    bf = nchw(b.float()).requires_grad_(True)
    wtr = wt.clone().requires_grad_(True)
    btr = bt.clone().requires_grad_(True)
    war = wa.clone().requires_grad_(True)
    u = F.conv_transpose2d(bf, wtr.permute(3, 2, 0, 1), btr, stride=2)
    z = F.conv2d(torch.cat([u, nchw(skip.float())], 1), war.permute(3, 2, 0, 1), padding=1)
    gb, gwt, gbt, gwa = torch.autograd.grad(z, (bf, wtr, btr, war), nchw(dz.float()))
    if with_wa:
        return nhwc(gb) * (b.float() > 0), gwt, gbt, gwa
    return nhwc(gb) * (b.float() > 0), gwt, gbt


@pytest.mark.parametrize("N,H,K,Cc,Cs,O", [(2, 64, 64, 32, 32, 32), (2, 32, 128, 64, 64, 64),
                                            (3, 16, 64, 32, 32, 32), (1, 32, 64, 32, 0, 32)])
def test_composite_tconv_dgrad(cuda_dev, N, H, K, Cc, Cs, O):
    """db = S2D(dz) (*) compose(Wt, Wa), masked by the ReLU bits of b -- vs autograd."""
    b, skip, wt, bt, wa, dz = _problem(cuda_dev, N, H, K, Cc, Cs, O, 11)
    ref_db, _, _ = _reference(b, skip, wt, bt, wa, dz)
    rs = (36 * O + 63) // 64 * 64
    wg = torch.empty(K, rs, device=cuda_dev, dtype=torch.bfloat16)
    C().generic("tconv_compose", [ptr(wt.reshape(4, Cc, K).contiguous()), ptr(wa.contiguous()), ptr(wg)],
                [Cc, K, O, Cc + Cs, rs], [], stream())
    bits = pack_bits(b)
    db = torch.empty(N, H, H, K, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=4 * O, s2d=O, src1=ptr(dz), wgt=ptr(wg),
                      Cout=K, dst1=ptr(db), mask1=ptr(bits), mask_bits=1), stream())
    torch.cuda.synchronize()
    assert rel_err(db, ref_db) < 2e-2


@pytest.mark.parametrize("N,H,K,Cc,Cs,O,splits,win", [(2, 64, 64, 32, 32, 32, 8, 0), (2, 64, 64, 32, 32, 32, 8, -1),
                                                       (2, 32, 128, 64, 64, 64, 5, 0), (3, 32, 32, 32, 32, 32, 7, 0),
                                                       (2, 32, 128, 64, 64, 64, 70, 0), (3, 16, 64, 32, 32, 32, 3, 0),
                                                       (3, 16, 64, 32, 32, 32, 3, -1), (2, 16, 128, 64, 64, 64, 5, 0),
                                                       (2, 128, 128, 64, 64, 64, 6, 0)])
def test_composite_tconv_weight_grads(cuda_dev, N, H, K, Cc, Cs, O, splits, win):
    """4x4-tap stride-2 slab sums H / per-tap bias sums Bs (coarse rows 16..128 wide: the
    window kernel -- at 16 a 32-pixel step spans two coarse rows, at 128 a window is one
    coarse row --, win -1: the tiled kernel) -> chain rule -> dWt, dbt."""
    b, skip, wt, bt, wa, dz = _problem(cuda_dev, N, H, K, Cc, Cs, O, 12)
    _, ref_wt, ref_bt, ref_wa = _reference(b, skip, wt, bt, wa, dz, with_wa=True)
    dev = cuda_dev
    slab = torch.zeros(splits * 16 * O * K, device=dev)
    bslab = torch.zeros(splits * 16 * O, device=dev)
    C().wgrad(dict(N=N, QD=1, QH=H, QW=H, AD=1, AH=2 * H, AW=2 * H, KD=1, KH=4, KW=4, stride=2, pad=1,
                   a1=ptr(dz), b=ptr(b), M1=O, M2=0, Nc=K, splits=splits, slab=ptr(slab), bias_slab=ptr(bslab),
                   bias_mode=2, win=win), stream())
    Hs = torch.zeros(16 * O * K, device=dev)
    Bs = torch.zeros(16 * O, device=dev)
    stage = torch.zeros(C().wgrad_reduce_stage_floats(max(splits, 64), 16, O, K) + 4096, device=dev)
    C().generic("wgrad_reduce", [ptr(slab), ptr(Hs), ptr(stage)], [splits, 16, O, O, K], [1.0], stream())
    C().generic("wgrad_reduce", [ptr(bslab), ptr(Bs), ptr(stage)], [splits, 1, 1, 1, 16 * O], [1.0], stream())
    # the slab sums themselves: H[sh][sw][o][k] = sum_{h,w} dz[2h + sh - 1][2w + sw - 1][o] b[h][w][k]
    dzp = F.pad(dz.float(), (0, 0, 1, 3, 1, 3))               # fine rows / cols -1 .. 2H + 1
    for sh in range(4):
        for sw in range(4):
            sl = dzp[:, sh:sh + 2 * H:2, sw:sw + 2 * H:2, :]
            ref_h = torch.einsum("nhwo,nhwk->ok", sl, b.float())
            got = Hs.view(16, O, K)[sh * 4 + sw]
            assert rel_err(got, ref_h) < 1e-3, (sh, sw)
            assert rel_err(Bs.view(16, O)[sh * 4 + sw], sl.sum((0, 1, 2))) < 1e-3, (sh, sw)
    dwt = torch.zeros(4, Cc, K, device=dev)
    dbt = torch.zeros(Cc, device=dev)
    C().generic("tconv_chain", [ptr(Hs), ptr(Bs), ptr(wa.contiguous()), ptr(dwt), ptr(dbt)], [Cc, K, O, Cc + Cs], [],
                stream())
    torch.cuda.synchronize()
    assert rel_err(dwt, ref_wt.reshape(4, Cc, K)) < 1e-3
    assert rel_err(dbt, ref_bt) < 1e-3
    # the consumer conv's weight gradient without its u half: the u rows from
    # H / Bs through Wt, bt; the skip rows copied from their own gradient
    dwa = torch.full((3, 3, Cc + Cs, O), float("nan"), device=dev)
    skg = ref_wa[:, :, Cc:, :].contiguous()
    C().generic("tconv_chain", [ptr(Hs), ptr(Bs), ptr(wa.contiguous()), ptr(dwt), ptr(dbt),
                                ptr(wt.reshape(4, Cc, K).contiguous()), ptr(bt), ptr(skg), ptr(dwa)],
                [Cc, K, O, Cc + Cs], [], stream())
    torch.cuda.synchronize()
    assert rel_err(dwa, ref_wa) < 1e-3
    assert torch.equal(dwa[:, :, Cc:, :], skg)



def _pad64(m):
    k = m.shape[1]
    out = torch.zeros(m.shape[0], (k + 63) // 64 * 64, dtype=m.dtype, device=m.device)
    out[:, :k] = m
    return out


@pytest.mark.parametrize("N,H,K,Cc,Cs,O,epi", [(2, 64, 64, 32, 32, 32, "fwd"), (2, 32, 128, 64, 64, 64, "fwd"),
                                                (3, 16, 64, 32, 32, 64, "fwd"), (2, 64, 64, 32, 32, 32, "stats"),
                                                (2, 32, 128, 64, 64, 64, "generic"), (2, 32, 32, 32, 32, 32, "fwd")])
def test_tconv_onload_forward(cuda_dev, N, H, K, Cc, Cs, O, epi):
    """Decoder forward z = conv3x3([tconv(b) + bt, skip]) with u formed on load from the
    coarse b (conv_win.h XF 5, fine rows 32..128 wide): bit-identical to the
    materialised tconv_fwd + concat conv (same MFMA operands and order), and vs fp32
    ATen conv_transpose2d + conv2d.  epi: ReLU forward with bits, normalisation
    statistics (pre-norm z), dropout (generic epilogue)."""
    b, skip, wt, bt, wa, _ = _problem(cuda_dev, N, H, K, Cc, Cs, O, 21)
    dev = cuda_dev
    F2 = 2 * H
    wtp = _pad64(wt.reshape(4 * Cc, K).bfloat16())                      # [tap][co] rows, K padded
    wap = _pad64(wa.bfloat16().permute(3, 0, 1, 2).reshape(O, 9 * (Cc + Cs)))
    ba = torch.randn(O, device=dev) * 0.1
    u = torch.empty(N, F2, F2, Cc, device=dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, C1=K, src1=ptr(b), wgt=ptr(wtp), bias=ptr(bt), Cout=4 * Cc,
                      shuffle=2, dst1=ptr(u)), stream())
    base = dict(N=N, OH=F2, OW=F2, IH=F2, IW=F2, KH=3, KW=3, pad=1, C1=Cc, C2=Cs, src2=ptr(skip), wgt=ptr(wap),
                bias=ptr(ba), Cout=O)
    outs = []
    for onload in (False, True):
        z = torch.full((N, F2, F2, O), float("nan"), device=dev, dtype=torch.bfloat16)
        d = dict(base, dst1=ptr(z))
        extra = []
        if epi == "fwd":
            bits = torch.zeros(N * F2 * F2 * O // 8, device=dev, dtype=torch.uint8)
            d.update(relu=1, relu_bits=ptr(bits))
            extra.append(bits)
        elif epi == "stats":
            rows, _ = C().conv_stat_tiles(dict(d, src1=1, stats=1))
            st = torch.zeros(rows * 2 * O, device=dev)
            d.update(stats=ptr(st))
            extra.append(st)
        else:
            d.update(relu=1, drop_rate=0.25, seed=7, salt=3)
        if onload:
            d.update(src1=ptr(b), ut_x=ptr(b), ut_w=ptr(wtp), ut_b=ptr(bt), ut_C=K, ut_kpad=wtp.shape[1])
        else:
            d.update(src1=ptr(u))
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append([z] + extra)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    ref_u = F.conv_transpose2d(nchw(b.float()), wt.bfloat16().float().permute(3, 2, 0, 1), bt, stride=2)
    ref = F.conv2d(torch.cat([ref_u, nchw(skip.float())], 1), wa.bfloat16().float().permute(3, 2, 0, 1), ba,
                   padding=1)
    z = outs[1][0].float()
    if epi == "fwd":
        assert rel_err(z, nhwc(F.relu(ref))) < 2e-2
    elif epi == "stats":
        assert rel_err(z, nhwc(ref)) < 2e-2
    else:
        kept = z != 0
        assert rel_err(z[kept] * 0.75, nhwc(F.relu(ref))[kept]) < 2e-2



@pytest.mark.parametrize("N,K,pf,rev", [(2, 64, 8, 0), (3, 64, 5, 1), (2, 32, 8, 1), (1, 64, 1, 0)])
def test_tconv_onload_persistent_window(cuda_dev, N, K, pf, rev):
    """conv9a's forward on the persistent tconv-on-load window (conv_win.h conv_win_pfu_kernel,
    win_pf > 0: 256-pixel windows, each wave forming one u halo row from its coarse row with
    tap-row weights held across the walk, the next window's coarse row and skip halo
    prefetched): bit-identical to the one-window XF 5 kernel -- output and ReLU bits."""
    H = 64
    b, skip, wt, bt, wa, _ = _problem(cuda_dev, N, H, K, 32, 32, 32, 22)
    dev = cuda_dev
    F2 = 2 * H
    wtp = _pad64(wt.reshape(4 * 32, K).bfloat16())
    wap = _pad64(wa.bfloat16().permute(3, 0, 1, 2).reshape(32, 9 * 64))
    ba = torch.randn(32, device=dev) * 0.1
    d0 = dict(N=N, OH=F2, OW=F2, IH=F2, IW=F2, KH=3, KW=3, pad=1, C1=32, C2=32, src1=ptr(b), src2=ptr(skip),
              wgt=ptr(wap), bias=ptr(ba), Cout=32, relu=1, ut_x=ptr(b), ut_w=ptr(wtp), ut_b=ptr(bt), ut_C=K,
              ut_kpad=wtp.shape[1], rev=rev)
    outs = []
    for p in (0, pf):
        z = torch.full((N, F2, F2, 32), float("nan"), device=dev, dtype=torch.bfloat16)
        bits = torch.zeros(N * F2 * F2 * 4, device=dev, dtype=torch.uint8)
        d = dict(d0, dst1=ptr(z), relu_bits=ptr(bits), win_pf=p)
        g = C().conv_fwd_grid(d)
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append((z, bits))
        if p:
            assert g == (N * F2 // 2 + p - 1) // p
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.isfinite(outs[1][0].float()).all()


@pytest.mark.parametrize("N,K,pf", [(2, 64, 8), (3, 32, 5)])
def test_tconv_onload_persistent_window_stats(cuda_dev, N, K, pf):
    """The normalised configs' conv9a forward on the persistent tconv-on-load window
    (statistics epilogue: pre-norm z + one {sum z, sum z^2} row per 256-pixel window):
    z bit-identical to the one-window XF 5 kernel, its per-512-pixel rows equal to the sums
    of row pairs, and the column sums equal to fp64 sums of z."""
    H = 64
    b, skip, wt, bt, wa, _ = _problem(cuda_dev, N, H, K, 32, 32, 32, 23)
    dev = cuda_dev
    F2 = 2 * H
    wtp = _pad64(wt.reshape(4 * 32, K).bfloat16())
    wap = _pad64(wa.bfloat16().permute(3, 0, 1, 2).reshape(32, 9 * 64))
    d0 = dict(N=N, OH=F2, OW=F2, IH=F2, IW=F2, KH=3, KW=3, pad=1, C1=32, C2=32, src1=ptr(b), src2=ptr(skip),
              wgt=ptr(wap), bias=0, Cout=32, relu=0, ut_x=ptr(b), ut_w=ptr(wtp), ut_b=ptr(bt), ut_C=K,
              ut_kpad=wtp.shape[1])
    outs = []
    for p in (0, pf):
        z = torch.full((N, F2, F2, 32), float("nan"), device=dev, dtype=torch.bfloat16)
        d = dict(d0, dst1=ptr(z), win_pf=p)
        rows, px = C().conv_stat_tiles(dict(d, stats=1))
        assert rows * px == N * F2 * F2 and px == (256 if p else 512)
        st = torch.full((rows * 2 * 32,), float("nan"), device=dev)
        d["stats"] = ptr(st)
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append((z, st.view(rows, 2, 32)))
    assert torch.equal(outs[0][0], outs[1][0])
    s_one, s_pf = outs[0][1], outs[1][1]
    assert torch.isfinite(s_pf).all()
    assert torch.allclose(s_pf.view(-1, 2, 2, 32).sum(1), s_one, rtol=1e-4, atol=1e-2)
    zf = outs[1][0].double().reshape(-1, 32)
    ref = torch.stack([zf.sum(0), (zf * zf).sum(0)])
    assert torch.allclose(s_pf.double().sum(0), ref, rtol=1e-4, atol=1e-1)
