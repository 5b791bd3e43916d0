"""The pipelined 8-wave row window (conv_pipe.h, default for 64-channel tiles on 2D rows
16..64 wide) against the 4-wave window kernel it replaces (tile 14) and the fp32 reference:
the per-element MFMA order is the same, so every stored tensor (outputs, ReLU bits, fused
pool values and codes, masked / routed data gradients, pre-norm z) is bit-identical; the
normalisation statistics rows are per tile (the tiles are twice as large) and their sums
agree to fp32 rounding."""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, _pack_bits, nchw, nhwc, pack_dgrad, pack_fwd, ptr, rel_err, stream

pytestmark = pytest.mark.gpu


def _pair(d, alloc):
    """Run conv dict `d` on the pipelined window (tile 12) and the 4-wave window (tile 14);
    alloc() -> (dict of fresh output pointers, tensors to compare)."""
    outs = []
    for tile in (12, 14):
        ptrs, ts = alloc()
        dd = dict(d, tile=tile, **ptrs)
        assert C().conv_fwd_grid(dd) > 0
        C().conv_fwd(dd, stream())
        torch.cuda.synchronize()
        outs.append(ts)
    return outs


@pytest.mark.parametrize("N,H,C1,C2,Cout,pool", [
    (3, 64, 64, 0, 64, True), (2, 64, 128, 0, 64, False), (2, 64, 64, 64, 64, False),
    (3, 32, 64, 0, 128, True), (2, 32, 128, 128, 128, False), (5, 32, 256, 0, 128, True),
    (4, 16, 128, 0, 256, True), (3, 16, 256, 256, 256, False), (2, 16, 64, 0, 64, False),
    (7, 16, 128, 0, 128, True)])
def test_conv_pipe_forward_matches_window_kernel(cuda_dev, N, H, C1, C2, Cout, pool):
    torch.manual_seed(N * 7 + H + C1 + C2)
    a = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    b2 = torch.randn(N, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.06).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
             src2=ptr(b2) if C2 else None, wgt=ptr(wp), bias=ptr(bias), Cout=Cout, relu=1)

    def alloc():
        y = torch.full((N, H, H, Cout), float("nan"), device=cuda_dev, dtype=torch.bfloat16)
        bits = torch.zeros(N * H * H * Cout // 8, device=cuda_dev, dtype=torch.uint8)
        p = dict(dst1=ptr(y), relu_bits=ptr(bits))
        ts = [y, bits]
        if pool:
            pooled = torch.empty(N, H // 2, H // 2, Cout, device=cuda_dev, dtype=torch.bfloat16)
            codes = torch.zeros(N * (H // 2) ** 2 * Cout // 8, device=cuda_dev, dtype=torch.int32)
            p.update(pool_dst=ptr(pooled), pool_code=ptr(codes))
            ts += [pooled, codes]
        return p, ts
    new, old = _pair(d, alloc)
    for x, y in zip(new, old):
        assert torch.equal(x, y)
    xin = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    ref = nhwc(F.relu(F.conv2d(xin, w.float().permute(3, 2, 0, 1), bias, padding=1)))
    assert rel_err(new[0], ref) < 1e-2
    assert torch.equal(new[1], _pack_bits(new[0]).reshape(-1))


@pytest.mark.parametrize("N,H,Co,C1,C2", [(2, 64, 64, 64, 64), (3, 32, 128, 128, 128), (3, 16, 256, 128, 128),
                                          (2, 32, 64, 128, 0), (4, 16, 128, 64, 0)])
def test_conv_pipe_dgrad_matches_window_kernel(cuda_dev, N, H, Co, C1, C2):
    """Data gradients: dual destination with bit masks (a decoder conv), and the skip half
    alone with the max-pool backward routed in its epilogue (route_gy)."""
    torch.manual_seed(H + Co + C1)
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.06).bfloat16()
    wdg = pack_dgrad(w)
    a1 = torch.randn(N, H, H, C1, device=cuda_dev)
    m1 = _pack_bits(a1)
    m2 = _pack_bits(torch.randn(N, H, H, max(C2, 8), device=cuda_dev))
    geo = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy), wgt=ptr(wdg))
    d = dict(geo, Cout=C1 + C2, D1=C1, mask1=ptr(m1), mask_bits=1)
    if C2:
        d.update(mask2=ptr(m2), mask_bits=3)

    def alloc():
        d1 = torch.full((N, H, H, C1), float("nan"), device=cuda_dev, dtype=torch.bfloat16)
        d2 = torch.full((N, H, H, max(C2, 1)), float("nan"), device=cuda_dev, dtype=torch.bfloat16)
        return dict(dst1=ptr(d1), dst2=ptr(d2) if C2 else None), [d1] + ([d2] if C2 else [])
    new, old = _pair(d, alloc)
    for x, y in zip(new, old):
        assert torch.equal(x, y)
    xr = torch.zeros(N, C1 + C2, H, H, device=cuda_dev, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1), xr, nchw(dy.float()))
    g = nhwc(g)
    assert rel_err(new[0], g[..., :C1] * (a1 > 0)) < 1e-2
    if C2:
        # the skip half alone with the pool backward in the epilogue
        y = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
        pooled = torch.empty(N, H // 2, H // 2, C2, device=cuda_dev, dtype=torch.bfloat16)
        codes = torch.zeros(N * (H // 2) ** 2 * C2 // 8, device=cuda_dev, dtype=torch.int32)
        C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, C2, 0], [], stream())
        dpool = torch.randn(N, H // 2, H // 2, C2, device=cuda_dev).bfloat16()
        bits = _pack_bits(y)
        ds = dict(geo, wgt=ptr(wdg) + 2 * C1 * wdg.shape[1], Cout=C2, mask1=ptr(bits), mask_bits=1,
                  route_gy=ptr(dpool), pool_code=ptr(codes))

        def alloc2():
            o = torch.full((N, H, H, C2), float("nan"), device=cuda_dev, dtype=torch.bfloat16)
            return dict(dst1=ptr(o)), [o]
        new2, old2 = _pair(ds, alloc2)
        assert torch.equal(new2[0], old2[0]) and torch.isfinite(new2[0].float()).all()


@pytest.mark.parametrize("N,H,Cin,Cout,C2", [(2, 64, 64, 64, 0), (3, 32, 128, 128, 128), (4, 16, 256, 256, 0)])
def test_conv_pipe_stats_epilogue(cuda_dev, N, H, Cin, Cout, C2):
    """Pre-normalisation forward: z bit-identical to the 4-wave window, per-tile {sum z,
    sum z^2} rows (twice the pixels per tile) summing to the same per-sample moments."""
    torch.manual_seed(3 + H)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    x2 = torch.randn(N, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin + C2, Cout, device=cuda_dev) * 0.06).bfloat16()
    b = torch.randn(Cout, device=cuda_dev)
    wp = pack_fwd(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, C2=C2, src1=ptr(x),
             src2=ptr(x2) if C2 else None, wgt=ptr(wp), bias=ptr(b), Cout=Cout, relu=0)
    res = []
    for tile in (12, 14):
        rows, px = C().conv_stat_tiles(dict(d, stats=1, tile=tile))
        assert rows * px == N * H * H and rows > 0
        z = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
        st = torch.full((rows, 2, Cout), float("nan"), device=cuda_dev)
        C().conv_fwd(dict(d, tile=tile, dst1=ptr(z), stats=ptr(st)), stream())
        torch.cuda.synchronize()
        res.append((z, st.view(N, rows // N, 2, Cout).sum(1), px))
    (z0, s0, px0), (z1, s1, px1) = res
    assert torch.equal(z0, z1)
    assert px0 == 2 * px1 or (H == 16 and px0 == px1)
    assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,H,Cg,Cy,gn,drop", [(2, 64, 64, 64, False, 0.0), (2, 32, 128, 128, True, 0.2),
                                               (4, 16, 256, 128, True, 0.0)])
def test_conv_pipe_dgrad_norm_epilogue(cuda_dev, N, H, Cg, Cy, gn, drop):
    torch.manual_seed(5 + H)
    dz = torch.randn(N, H, H, Cg, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cy, Cg, device=cuda_dev) * 0.06).bfloat16()
    z = torch.randn(N, H, H, Cy, device=cuda_dev).bfloat16()
    rows_c = N if gn else 1
    a = 0.5 + torch.rand(rows_c, Cy, device=cuda_dev)
    c = 0.3 * torch.randn(rows_c, Cy, device=cuda_dev)
    wp = pack_dgrad(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cg, src1=ptr(dz), wgt=ptr(wp), Cout=Cy, relu=0,
             nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=Cy if gn else 0, npix=H * H, nd_rate=drop, nd_salt=3, seed=77)
    res = []
    for tile in (12, 14):
        rows, px = C().conv_stat_tiles(dict(d, stats=1, tile=tile))
        g = torch.empty(N, H, H, Cy, device=cuda_dev, dtype=torch.bfloat16)
        st = torch.full((rows, 2, Cy), float("nan"), device=cuda_dev)
        C().conv_fwd(dict(d, tile=tile, dst1=ptr(g), stats=ptr(st)), stream())
        torch.cuda.synchronize()
        res.append((g, st.view(N, rows // N, 2, Cy).sum(1)))
    (g0, s0), (g1, s1) = res
    assert torch.equal(g0, g1)
    assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,H,K,O", [(2, 64, 64, 32), (2, 32, 128, 64), (3, 32, 64, 32)])
def test_conv_pipe_space_to_depth_dgrad(cuda_dev, N, H, K, O):
    """The composite transposed-conv data gradient (XF 4: space-to-depth source, zero taps
    skipped) on the pipelined window."""
    torch.manual_seed(9 + H)
    dz = torch.randn(N, 2 * H, 2 * H, O, device=cuda_dev).bfloat16()
    wg = (torch.randn(K, (36 * O + 63) // 64 * 64, device=cuda_dev) * 0.05).bfloat16()
    bits = _pack_bits(torch.randn(N, H, H, K, device=cuda_dev))
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=4 * O, s2d=O, src1=ptr(dz), wgt=ptr(wg), Cout=K,
             mask1=ptr(bits), mask_bits=1)

    def alloc():
        o = torch.full((N, H, H, K), float("nan"), device=cuda_dev, dtype=torch.bfloat16)
        return dict(dst1=ptr(o)), [o]
    new, old = _pair(d, alloc)
    assert torch.equal(new[0], old[0]) and torch.isfinite(new[0].float()).all()


def test_conv_pipe_reverse_order_and_tail_windows(cuda_dev):
    """rev = 1 and a batch whose row count is not a multiple of the window (N H % R != 0
    cannot happen: H % R == 0 by eligibility) -- odd N exercises the XCD remap tail."""
    torch.manual_seed(11)
    N, H, Ci, Co = 5, 32, 64, 64
    x = torch.randn(N, H, H, Ci, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Ci, Co, device=cuda_dev) * 0.08).bfloat16()
    b = torch.randn(Co, device=cuda_dev)
    wp = pack_fwd(w)
    outs = []
    for rev in (0, 1):
        y = torch.empty(N, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
        C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Ci, src1=ptr(x), wgt=ptr(wp),
                          bias=ptr(b), Cout=Co, relu=1, dst1=ptr(y), rev=rev), stream())
        torch.cuda.synchronize()
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    ref = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(outs[0], ref) < 1e-2


@pytest.mark.parametrize("N,H,C1,C2,Cout,splits", [
    (4, 64, 64, 0, 64, 3), (3, 64, 64, 64, 64, 9), (2, 64, 32, 0, 64, 2), (5, 32, 64, 0, 128, 4),
    (2, 32, 128, 128, 128, 3), (3, 32, 32, 0, 32, 40), (4, 16, 64, 0, 64, 3), (3, 16, 128, 128, 128, 5),
    (2, 16, 256, 0, 256, 70), (2, 64, 64, 0, 32, 4)])
def test_wgrad_pipe_matches_window_kernel(cuda_dev, N, H, C1, C2, Cout, splits):
    """The pipelined 8-wave window weight gradient (wgrad_pipe.hip, default on 16..64-wide
    rows) against the 4-wave window (win 2) and the fp32 autograd reference: kernel and
    fused bias sums, concat sources, more splits than windows (empty splits write zeros)."""
    from test_gpu_kernels import _wgrad
    torch.manual_seed(N + H + C1 + C2 + Cout + splits)
    a = F.relu(torch.randn(N, H, H, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(N, H, H, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(N, H, H, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=C1, M2=C2, a1=ptr(a),
             a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1)
    gw0, gb0 = _wgrad(dict(d, win=0), splits, 9, Mt, Mt, Cout, 9 * Mt * Cout, bias_w=(splits, Cout))
    gw2, gb2 = _wgrad(dict(d, win=2), splits, 9, Mt, Mt, Cout, 9 * Mt * Cout, bias_w=(splits, Cout))
    torch.cuda.synchronize()
    assert rel_err(gw0, gw2) < 1e-5 and rel_err(gb0, gb2) < 1e-5
    inp = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    w = torch.zeros(Cout, Mt, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(inp, w, bb, padding=1), [w, bb], nchw(dy.float()))
    assert rel_err(gw0, gwr.permute(2, 3, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb0, gbr) < 2e-3


@pytest.mark.parametrize("N,H,Cin,Cout,gn,stats", [(2, 64, 64, 64, False, True), (3, 32, 128, 128, True, True),
                                                   (4, 16, 256, 256, False, False), (2, 32, 64, 128, True, False)])
def test_conv_pipe_normalise_on_load(cuda_dev, N, H, Cin, Cout, gn, stats):
    """XF 1 (the input normalised on load, y = relu(a z + c), y of the window's own rows to
    xout) on the pipelined window: output, xout and statistics equal the 4-wave window's."""
    torch.manual_seed(17 + H)
    z = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    rows = N if gn else 1
    a = 0.5 + torch.rand(rows, Cin, device=cuda_dev)
    b = 0.3 * torch.randn(rows, Cin, device=cuda_dev)
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.06).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(z), wgt=ptr(wp), bias=ptr(bias),
             Cout=Cout, relu=0, xform=1, xa=ptr(a), xb=ptr(b), xcs=Cin if gn else 0)
    res = []
    for tile in (12, 14):
        out = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
        yo = torch.full_like(z, float("nan"))
        dd = dict(d, tile=tile, dst1=ptr(out), xout=ptr(yo))
        st = None
        if stats:
            nr, _ = C().conv_stat_tiles(dict(dd, stats=1))
            st = torch.zeros(nr, 2, Cout, device=cuda_dev)
            dd["stats"] = ptr(st)
        else:
            dd.update(relu=0, drop_rate=0.0, out_scale=1.0)
        C().conv_fwd(dd, stream())
        torch.cuda.synchronize()
        res.append((out, yo, None if st is None else st.view(N, -1, 2, Cout).sum(1)))
    (o0, y0, s0), (o1, y1, s1) = res
    assert torch.equal(o0, o1) and torch.equal(y0, y1) and torch.isfinite(y0.float()).all()
    if stats:
        assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)
    yr = torch.clamp(a.view(rows, 1, 1, Cin) * z.float() + b.view(rows, 1, 1, Cin), min=0).bfloat16()
    ref = nhwc(F.conv2d(nchw(yr.float()), w.float().permute(3, 2, 0, 1), bias, padding=1))
    assert rel_err(o0, ref) < 1e-2
