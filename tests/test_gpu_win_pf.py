"""Persistent prefetching row window (conv_win.h conv_win_pf_kernel, win_pf > 0): the
level-1 32 -> 32 channel convs on 128-wide rows -- bias + ReLU forward with the fused
max-pool, ReLU bits or segmentation head, and the data gradient with bit masks and the
fused pool backward -- write exactly what the one-window-per-workgroup kernel writes
(same operands, tap order and epilogue), for window counts that do and do not divide by
win_pf and in both walk orders."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, _pack_bits, nchw, nhwc, pack_dgrad, pack_fwd, ptr, rel_err, stream

pytestmark = pytest.mark.gpu
H = 128


def _fwd_run(x, wp, b, pf, rev, N, extra):
    y = torch.empty(N, H, H, 32, device=x.device, dtype=torch.bfloat16)
    bits = torch.zeros(N * H * H * 4, device=x.device, dtype=torch.uint8)
    pooled = torch.zeros(N, H // 2, H // 2, 32, device=x.device, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * 4, device=x.device, dtype=torch.int32)
    logit = torch.zeros(N * H * H, device=x.device)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(x), wgt=ptr(wp), bias=ptr(b),
             Cout=32, relu=1, dst1=ptr(y), win_pf=pf, rev=rev)
    if extra == "pool":
        d.update(pool_dst=ptr(pooled), pool_code=ptr(codes), relu_bits=ptr(bits))
    elif extra == "head":
        hw = (torch.arange(32, device=x.device, dtype=torch.float32) - 15.5) / 40.0
        hb = torch.tensor([0.25], device=x.device)
        d.update(head_w=ptr(hw), head_b=ptr(hb), head_logit=ptr(logit), relu_bits=ptr(bits))
        d["_keep"] = (hw, hb)
    grid = C().conv_fwd_grid({k: v for k, v in d.items() if k != "_keep"})
    C().conv_fwd({k: v for k, v in d.items() if k != "_keep"}, stream())
    torch.cuda.synchronize()
    return grid, (y, bits, pooled, codes, logit)


@pytest.mark.parametrize("N,pf,rev,extra", [(2, 16, 0, "pool"), (3, 5, 1, "pool"), (1, 1, 0, "head"),
                                            (5, 16, 1, "head"), (2, 7, 0, "none"), (4, 64, 0, "pool")])
def test_win_pf_forward_equals_window_kernel(cuda_dev, N, pf, rev, extra):
    torch.manual_seed(81)
    x = F.relu(torch.randn(N, H, H, 32, device=cuda_dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(32, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    g0, ref = _fwd_run(x, wp, b, 0, rev, N, extra)
    g1, out = _fwd_run(x, wp, b, pf, rev, N, extra)
    nwin = N * H // 4
    assert g0 == nwin and g1 == (nwin + pf - 1) // pf
    for a, bb in zip(ref, out):
        assert torch.equal(a, bb)
    exp = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(out[0], exp) < 1e-2
    if extra == "head":
        assert out[4].abs().sum() > 0


@pytest.mark.parametrize("N,pf,rev,route", [(2, 16, 0, True), (3, 3, 1, True), (2, 16, 1, False), (1, 64, 0, False)])
def test_win_pf_dgrad_equals_window_kernel(cuda_dev, N, pf, rev, route):
    torch.manual_seed(82)
    y = F.relu(torch.randn(N, H, H, 32, device=cuda_dev)).bfloat16()        # the skip source (mask)
    pooled = torch.empty(N, H // 2, H // 2, 32, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * 4, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, 32, 0], [], stream())
    dpool = torch.randn(N, H // 2, H // 2, 32, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    dy = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
    bits = _pack_bits(y)
    wd = pack_dgrad(w)
    outs = []
    for p in (0, pf):
        dx = torch.empty(N, H, H, 32, device=cuda_dev, dtype=torch.bfloat16)
        d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(dy), wgt=ptr(wd),
                 Cout=32, dst1=ptr(dx), win_pf=p, rev=rev)
        if route:
            d.update(mask1=ptr(bits), mask_bits=1, route_gy=ptr(dpool), pool_code=ptr(codes))
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append(dx)
    assert torch.equal(outs[0], outs[1])
    if not route:
        exp = nhwc(F.conv_transpose2d(nchw(dy.float()), w.float().permute(3, 2, 0, 1), padding=1))
        assert rel_err(outs[1], exp) < 1e-2


def test_win_pf_not_taken_off_shape(cuda_dev):
    """win_pf only changes the launch on its shape: 64-wide rows / 64 channels keep the
    one-window grid."""
    for OW, Cin, Cout in ((64, 32, 32), (128, 64, 32), (128, 32, 64)):
        d = dict(N=2, OH=OW, OW=OW, IH=OW, IW=OW, KH=3, KW=3, pad=1, C1=Cin, Cout=Cout, relu=1, src1=1, wgt=1,
                 dst1=1, win_pf=16)
        assert C().conv_fwd_grid(d) == C().conv_fwd_grid(dict(d, win_pf=0))


@pytest.mark.parametrize("mode", ["stats", "dropout", "dgrad_norm_bn", "dgrad_norm_gn"])
def test_win_pf_other_epilogues_equal_window_kernel(cuda_dev, mode):
    """Statistics forward (norm configs), generic dropout forward and the data gradient of
    a normalised activation: the persistent window writes the same outputs and the same
    per-window statistics rows."""
    torch.manual_seed(83)
    N = 3
    x = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(32, device=cuda_dev) * 0.1
    z = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
    gn = mode == "dgrad_norm_gn"
    a = torch.rand(N if gn else 1, 32, device=cuda_dev) + 0.5
    c = torch.randn(N if gn else 1, 32, device=cuda_dev) * 0.1
    wp, wd = pack_fwd(w), pack_dgrad(w)
    outs = []
    for pf in (0, 8):
        y = torch.empty(N, H, H, 32, device=cuda_dev, dtype=torch.bfloat16)
        d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(x), Cout=32, dst1=ptr(y),
                 win_pf=pf)
        if mode == "stats":
            d.update(wgt=ptr(wp), bias=ptr(b))
        elif mode == "dropout":
            d.update(wgt=ptr(wp), bias=ptr(b), relu=1, drop_rate=0.3, seed=7, salt=2)
        else:
            d.update(wgt=ptr(wd), relu=0, nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=32 if gn else 0, npix=H * H,
                     nd_rate=0.2, nd_salt=4, seed=9)
        st = None
        if mode != "dropout":
            rows, _ = C().conv_stat_tiles(dict(d, stats=1))
            assert rows == N * H // 4
            st = torch.full((rows * 2 * 32,), float("nan"), device=cuda_dev)
            d["stats"] = ptr(st)
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append((y, st))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.isfinite(outs[1][1]).all() and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,pf,rev,bce", [(3, 8, 0, 0.0), (2, 5, 1, 0.5)])
def test_win_pf_head_onload_dgrad_equals_window_kernel(cuda_dev, N, pf, rev, bce):
    """Head-on-load data gradient (XF 3, dgrad:conv9b): the persistent window forms the
    same dY halo from the prefetched probability / target / ReLU bits."""
    torch.manual_seed(84)
    P = N * H * H
    x = F.relu(torch.randn(N, H, H, 32, device=cuda_dev)).bfloat16()
    hw = torch.randn(32, device=cuda_dev) * 0.3
    prob = torch.rand(P, device=cuda_dev) * 0.98 + 0.01
    t = (torch.rand(P, device=cuda_dev) > 0.6).bfloat16()
    sums = torch.stack([(t.float() * prob).sum(), t.float().sum(), prob.sum(), torch.zeros((), device=cuda_dev)])
    gsc = torch.full((1,), 2.0, device=cuda_dev)
    pos = (x.reshape(P, 4, 8).float() > 0).to(torch.int32)
    xbits = (pos << torch.arange(8, device=cuda_dev, dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()
    a9 = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
    a9b = _pack_bits(a9)
    wt = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    wd = pack_dgrad(wt)
    outs = []
    for p in (0, pf):
        dx = torch.full_like(a9, float("nan"))
        C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(x), wgt=ptr(wd), Cout=32,
                          mask1=ptr(a9b), mask_bits=1, dst1=ptr(dx), win_pf=p, rev=rev, hg_prob=ptr(prob),
                          hg_t=ptr(t), hg_sums=ptr(sums), hg_w=ptr(hw), hg_bits=ptr(xbits), hg_gscale=ptr(gsc),
                          hg_inv_total=1.0 / P, hg_bce_w=bce), stream())
        torch.cuda.synchronize()
        outs.append(dx)
    assert torch.isfinite(outs[1]).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,HW,pf,rev,mode", [(1, 256, 8, 0, "pool"), (2, 256, 3, 1, "dgrad"), (1, 512, 8, 1, "pool"),
                                              (1, 512, 5, 0, "dgrad"), (1, 512, 8, 0, "stats")])
def test_win_pf_segmented_rows_equal_window_kernel(cuda_dev, N, HW, pf, rev, mode):
    """Rows wider than 128 (the 512^2 / 256^2 models' level 1) as 128-wide segments: the
    halo columns -1 / 128 come from the neighbouring segments."""
    torch.manual_seed(85)
    x = F.relu(torch.randn(N, HW, HW, 32, device=cuda_dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(32, device=cuda_dev) * 0.1
    geo = dict(N=N, OH=HW, OW=HW, IH=HW, IW=HW, KH=3, KW=3, pad=1, C1=32, Cout=32, rev=rev)
    y = torch.empty(N, HW, HW, 32, device=cuda_dev, dtype=torch.bfloat16)
    if mode == "pool":
        bits = torch.empty(N * HW * HW * 4, device=cuda_dev, dtype=torch.uint8)
        pooled = torch.empty(N, HW // 2, HW // 2, 32, device=cuda_dev, dtype=torch.bfloat16)
        codes = torch.empty(N * (HW // 2) ** 2 * 4, device=cuda_dev, dtype=torch.int32)
        wp = pack_fwd(w)
        d = dict(geo, src1=ptr(x), wgt=ptr(wp), bias=ptr(b), relu=1, dst1=ptr(y), relu_bits=ptr(bits),
                 pool_dst=ptr(pooled), pool_code=ptr(codes))
        outs = [y, bits, pooled, codes]
    elif mode == "stats":
        wp = pack_fwd(w)
        d = dict(geo, src1=ptr(x), wgt=ptr(wp), bias=ptr(b), dst1=ptr(y))
        rows, _ = C().conv_stat_tiles(dict(d, stats=1))
        st = torch.empty(rows * 2 * 32, device=cuda_dev)
        d["stats"] = ptr(st)
        outs = [y, st]
    else:
        wp = pack_dgrad(w)
        mk = _pack_bits(torch.randn(N, HW, HW, 32, device=cuda_dev))
        d = dict(geo, src1=ptr(x), wgt=ptr(wp), dst1=ptr(y), mask1=ptr(mk), mask_bits=1)
        outs = [y]
    res = []
    for p in (0, pf):
        for t in outs:
            t.fill_(float("nan") if t.is_floating_point() else 0)
        g = C().conv_fwd_grid(dict(d, win_pf=p))
        C().conv_fwd(dict(d, win_pf=p), stream())
        torch.cuda.synchronize()
        res.append([t.clone() for t in outs])
        if p:
            nwin = N * HW // 4 * (HW // 128)
            assert g == (nwin + p - 1) // p
    for a, bb in zip(*res):
        assert torch.equal(a, bb)
    if mode == "pool":
        exp = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
        assert rel_err(res[1][0], exp) < 1e-2


@pytest.mark.parametrize("N,pf,rev,gn,stats", [(3, 8, 0, False, True), (2, 5, 1, True, True), (2, 8, 0, True, False)])
def test_win_pf_normalise_on_load_equals_window_kernel(cuda_dev, N, pf, rev, gn, stats):
    """Normalised-input convs (norm configs' conv1b / conv9b, xform 1): the persistent
    window applies y = relu(a z + b) to the prefetched halo in registers and writes the
    window's own rows to xout -- the same conv output, statistics rows and y."""
    torch.manual_seed(86)
    z = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
    a = torch.rand(N if gn else 1, 32, device=cuda_dev) + 0.5
    b = torch.randn(N if gn else 1, 32, device=cuda_dev) * 0.2
    w = (torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()
    bias = torch.randn(32, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    out = torch.empty(N, H, H, 32, device=cuda_dev, dtype=torch.bfloat16)
    yo = torch.empty_like(z)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(z), wgt=ptr(wp), bias=ptr(bias),
             Cout=32, relu=0, dst1=ptr(out), xform=1, xa=ptr(a), xb=ptr(b), xcs=32 if gn else 0, xout=ptr(yo), rev=rev)
    outs = [out, yo]
    if stats:
        nr, _ = C().conv_stat_tiles(dict(d, stats=1))
        st = torch.empty(nr * 2 * 32, device=cuda_dev)
        d["stats"] = ptr(st)
        outs.append(st)
    else:
        d.update(relu=1, drop_rate=0.2, seed=3, salt=7)
    res = []
    for p in (0, pf):
        for t in outs:
            t.fill_(float("nan"))
        C().conv_fwd(dict(d, win_pf=p), stream())
        torch.cuda.synchronize()
        res.append([t.clone() for t in outs])
    for x0, x1 in zip(*res):
        assert torch.equal(x0, x1)
    y_ref = F.relu(z.float() * (a[:, None, None, :] if gn else a) + (b[:, None, None, :] if gn else b))
    assert (res[1][1].float() - y_ref).abs().max() <= 1e-2 * y_ref.abs().max()
