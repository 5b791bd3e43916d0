"""Chunk-pipelined row window (conv_win.h conv_win_cp_kernel, win_cp = 1): the 64-channel
windows of 64-wide rows with two or more input chunks (other row widths keep the DMA
chunk loop: the cases there check that win_cp leaves them unchanged) -- forward (bias + ReLU, fused
max-pool, ReLU bits, statistics, dropout), data gradient (two destinations, bit masks,
fused pool backward, the normalised-activation epilogue), plain and concat sources, both
walk orders -- write exactly what conv_win_kernel writes (same LDS images, operands, tap
order and epilogue)."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, _pack_bits, nchw, nhwc, pack_dgrad, pack_fwd, ptr, rel_err, stream

pytestmark = pytest.mark.gpu


def _run(d, outs):
    res = []
    for cp in (0, 2):
        for t in outs:
            t.fill_(float("nan") if t.is_floating_point() else 0)
        C().conv_fwd(dict(d, win_cp=cp), stream())
        torch.cuda.synchronize()
        res.append([t.clone() for t in outs])
    for a, b in zip(*res):
        assert torch.equal(a, b)
    return res[1]


@pytest.mark.parametrize("N,H,C1,C2,Cout,rev", [(3, 64, 64, 0, 64, 0), (2, 64, 32, 32, 64, 1), (4, 32, 128, 0, 128, 0),
                                                 (3, 32, 64, 64, 128, 1), (8, 16, 256, 0, 256, 0),
                                                 (5, 16, 128, 128, 128, 1), (2, 64, 64, 64, 64, 0)])
def test_win_cp_forward_equals_window_kernel(cuda_dev, N, H, C1, C2, Cout, rev):
    torch.manual_seed(91)
    x1 = F.relu(torch.randn(N, H, H, C1, device=cuda_dev)).bfloat16()
    x2 = F.relu(torch.randn(N, H, H, max(C2, 1), device=cuda_dev)).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.05).bfloat16()
    b = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    y = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    bits = torch.empty(N * H * H * Cout // 8, device=cuda_dev, dtype=torch.uint8)
    pooled = torch.empty(N, H // 2, H // 2, Cout, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.empty(N * (H // 2) ** 2 * Cout // 8, device=cuda_dev, dtype=torch.int32)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(x1), wgt=ptr(wp), bias=ptr(b),
             Cout=Cout, relu=1, dst1=ptr(y), relu_bits=ptr(bits), rev=rev)
    outs = [y, bits]
    if C2:
        d["src2"] = ptr(x2)
    else:
        d.update(pool_dst=ptr(pooled), pool_code=ptr(codes))
        outs += [pooled, codes]
    got = _run(d, outs)
    xin = torch.cat([x1, x2], -1) if C2 else x1
    exp = nhwc(F.relu(F.conv2d(nchw(xin.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(got[0], exp) < 1e-2


@pytest.mark.parametrize("mode", ["stats", "dropout"])
@pytest.mark.parametrize("H", [16, 32, 64])
def test_win_cp_stats_and_dropout_forward(cuda_dev, mode, H):
    torch.manual_seed(92)
    N, Cin, Cout = 4, 128, 64
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.05).bfloat16()
    b = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    y = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp), bias=ptr(b),
             Cout=Cout, dst1=ptr(y))
    outs = [y]
    if mode == "stats":
        rows, _ = C().conv_stat_tiles(dict(d, stats=1))
        st = torch.empty(rows * 2 * Cout, device=cuda_dev)
        d["stats"] = ptr(st)
        outs.append(st)
    else:
        d.update(relu=1, drop_rate=0.25, seed=3, salt=5)
    _run(d, outs)


@pytest.mark.parametrize("N,H,C1,C2,Co", [(2, 64, 64, 64, 64), (4, 32, 128, 128, 128), (4, 16, 256, 256, 256)])
def test_win_cp_dgrad_dual_dest_and_pool_route(cuda_dev, N, H, C1, C2, Co):
    """dY -> (upsampled half, skip half) with bit masks, then the skip half alone with the
    fused pool backward (the decoder's deferred skip data gradient)."""
    torch.manual_seed(93)
    y = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
    pooled = torch.empty(N, H // 2, H // 2, C2, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * C2 // 8, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, C2, 0], [], stream())
    dpool = torch.randn(N, H // 2, H // 2, C2, device=cuda_dev).bfloat16()
    m1 = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.05).bfloat16()
    wdg = pack_dgrad(w)
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    b1, b2 = _pack_bits(m1), _pack_bits(y)
    geo = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy))
    d1 = torch.empty(N, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    _run(dict(geo, wgt=ptr(wdg), Cout=C1 + C2, D1=C1, dst1=ptr(d1), dst2=ptr(d2), mask1=ptr(b1), mask2=ptr(b2),
              mask_bits=3, mask_scale2=1.25), [d1, d2])
    ds = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    _run(dict(geo, wgt=ptr(wdg) + 2 * C1 * wdg.shape[1], Cout=C2, dst1=ptr(ds), mask1=ptr(b2), mask_bits=1,
              route_gy=ptr(dpool), pool_code=ptr(codes)), [ds])
    assert ds.float().abs().sum() > 0


@pytest.mark.parametrize("gn", [False, True])
def test_win_cp_dgrad_norm(cuda_dev, gn):
    torch.manual_seed(94)
    N, H, Ci, Cy = 4, 32, 128, 64
    z = torch.randn(N, H, H, Cy, device=cuda_dev).bfloat16()
    a = torch.rand(N if gn else 1, Cy, device=cuda_dev) + 0.5
    c = torch.randn(N if gn else 1, Cy, device=cuda_dev) * 0.1
    w = (torch.randn(3, 3, Cy, Ci, device=cuda_dev) * 0.05).bfloat16()     # forward Cy -> Ci (HWIO)
    wdg = pack_dgrad(w)
    dy = torch.randn(N, H, H, Ci, device=cuda_dev).bfloat16()
    g = torch.empty(N, H, H, Cy, device=cuda_dev, dtype=torch.bfloat16)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Ci, src1=ptr(dy), wgt=ptr(wdg), Cout=Cy, relu=0,
             dst1=ptr(g), nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=Cy if gn else 0, npix=H * H, nd_rate=0.2, nd_salt=4,
             seed=9)
    rows, _ = C().conv_stat_tiles(dict(d, stats=1))
    st = torch.empty(rows * 2 * Cy, device=cuda_dev)
    _run(dict(d, stats=ptr(st)), [g, st])


def _pad64(m):
    kp = (m.shape[1] + 63) // 64 * 64
    out = torch.zeros(m.shape[0], kp, dtype=m.dtype, device=m.device)
    out[:, :m.shape[1]] = m
    return out


@pytest.mark.parametrize("N,D,C1,C2,Cout,rev", [(1, 4, 32, 0, 32, 0), (2, 3, 32, 32, 32, 1), (1, 2, 64, 0, 64, 0),
                                                (1, 5, 32, 32, 64, 0)])
def test_win_cp128_3d_equals_window_kernel(cuda_dev, N, D, C1, C2, Cout, rev):
    """3D level 1 (3x3x3 on 128-wide rows): items = depth taps x chunks; forward with ReLU
    bits and statistics, concat data gradient with two destinations and a bit mask."""
    torch.manual_seed(95)
    H = 128
    a = torch.randn(N, D, H, H, C1, device=cuda_dev).bfloat16()
    b2 = torch.randn(N, D, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, 3, C1 + C2, Cout, device=cuda_dev) * 0.05).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = _pad64(w.permute(4, 0, 1, 2, 3).reshape(Cout, -1))
    geo = dict(N=N, OD=D, OH=H, OW=H, ID=D, IH=H, IW=H, KD=3, KH=3, KW=3, pad=1, rev=rev)
    out = torch.empty(N, D, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    bits = torch.empty(N * D * H * H * Cout // 8, device=cuda_dev, dtype=torch.uint8)
    d = dict(geo, C1=C1, C2=C2, src1=ptr(a), wgt=ptr(wp), bias=ptr(bias), Cout=Cout, relu=1, dst1=ptr(out),
             relu_bits=ptr(bits))
    if C2:
        d["src2"] = ptr(b2)
    got = _run(d, [out, bits])
    xin = torch.cat([a, b2], -1) if C2 else a
    ref = F.relu(F.conv3d(xin.float().permute(0, 4, 1, 2, 3), w.float().permute(4, 3, 0, 1, 2), bias, padding=1))
    assert rel_err(got[0], ref.permute(0, 2, 3, 4, 1)) < 1e-2
    z = torch.empty_like(out)
    ds = dict(geo, C1=C1, C2=C2, src1=ptr(a), wgt=ptr(wp), bias=ptr(bias), Cout=Cout, dst1=ptr(z))
    if C2:
        ds["src2"] = ptr(b2)
    rows, _ = C().conv_stat_tiles(dict(ds, stats=1))
    st = torch.empty(rows * 2 * Cout, device=cuda_dev)
    ds["stats"] = ptr(st)
    _run(ds, [z, st])
    dy = torch.randn(N, D, H, H, Cout, device=cuda_dev).bfloat16()
    wdg = _pad64(w.flip(0, 1, 2).permute(3, 0, 1, 2, 4).reshape(C1 + C2, -1))
    d1 = torch.empty(N, D, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, D, H, H, max(C2, 1), device=cuda_dev, dtype=torch.bfloat16)
    b2b = _pack_bits(b2) if C2 else None
    dd = dict(geo, C1=Cout, src1=ptr(dy), wgt=ptr(wdg), Cout=C1 + C2, D1=C1, dst1=ptr(d1))
    if C2:
        dd.update(dst2=ptr(d2), mask2=ptr(b2b), mask_bits=2)
    _run(dd, [d1, d2] if C2 else [d1])


@pytest.mark.parametrize("N,C1,C2,Cout,rev", [(2, 64, 0, 32, 0), (2, 32, 32, 32, 1), (1, 128, 0, 64, 0),
                                              (1, 128, 128, 128, 1)])
def test_win_cp128_2d_multichunk_equals_window_kernel(cuda_dev, N, C1, C2, Cout, rev):
    """2D 128-wide rows with two or more input chunks (the 512^2 model's 128-wide level,
    concat decoder convs): forward with pool + bits, data gradient."""
    torch.manual_seed(96)
    H = 128
    x1 = F.relu(torch.randn(N, H, H, C1, device=cuda_dev)).bfloat16()
    x2 = F.relu(torch.randn(N, H, H, max(C2, 1), device=cuda_dev)).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.05).bfloat16()
    b = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    y = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    bits = torch.empty(N * H * H * Cout // 8, device=cuda_dev, dtype=torch.uint8)
    pooled = torch.empty(N, H // 2, H // 2, Cout, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.empty(N * (H // 2) ** 2 * Cout // 8, device=cuda_dev, dtype=torch.int32)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(x1), wgt=ptr(wp), bias=ptr(b),
             Cout=Cout, relu=1, dst1=ptr(y), relu_bits=ptr(bits), rev=rev)
    outs = [y, bits]
    if C2:
        d["src2"] = ptr(x2)
    else:
        d.update(pool_dst=ptr(pooled), pool_code=ptr(codes))
        outs += [pooled, codes]
    got = _run(d, outs)
    xin = torch.cat([x1, x2], -1) if C2 else x1
    exp = nhwc(F.relu(F.conv2d(nchw(xin.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(got[0], exp) < 1e-2
    dy = torch.randn(N, H, H, Cout, device=cuda_dev).bfloat16()
    wdg = pack_dgrad(w)
    dx = torch.empty(N, H, H, C1 + C2, device=cuda_dev, dtype=torch.bfloat16)
    if Cout >= 64:
        _run(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cout, src1=ptr(dy), wgt=ptr(wdg), Cout=C1 + C2,
                  dst1=ptr(dx), rev=rev), [dx])
