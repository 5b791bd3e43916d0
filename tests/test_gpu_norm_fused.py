"""Fused Conv + BatchNorm/GroupNorm epilogues (conv_epilogue.h EPI_STATS /
EPI_DGRAD_NORM) against fp32 PyTorch references.

* forward: the conv writes the pre-norm z and per-tile {sum z, sum z^2} rows; the
  rows of every tile sum to the reference moments (per sample when the tiles are
  per-sample, which GroupNorm needs);
* data gradient: the ReLU / dropout mask of y = dropout(relu(a z + c)) is
  recomputed from z, and the tile rows sum to {sum g, sum g z}.

The row-window, first-layer, implicit-GEMM and transposed-conv kernels are all
covered (shapes pick each kernel).
"""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, nchw, nhwc, pack_dgrad, pack_fwd, ptr, rel_err, stream

pytestmark = pytest.mark.gpu


def _moments(z):            # z: [N, H, W, C] -> per-sample [N, 2, C]
    zf = z.float().reshape(z.shape[0], -1, z.shape[-1])
    return torch.stack([zf.sum(1), (zf * zf).sum(1)], 1)


@pytest.mark.parametrize("N,H,Cin,Cout,C2,tile", [
    (2, 128, 32, 32, 0, 0),      # row window, 128-wide rows
    (4, 16, 64, 64, 0, 0),       # row window, 16-wide rows
    (2, 32, 32, 64, 32, 0),      # row window, concat source
    (8, 8, 128, 256, 0, 0),      # implicit GEMM (8-wide rows), tiles span samples
    (2, 64, 4, 32, 0, 0),        # first-layer window kernel
    (2, 256, 32, 32, 0, 0),      # segmented 128-wide windows
    (2, 128, 32, 64, 0, 12),     # 64-channel row window (256-pixel windows)
    (4, 16, 64, 128, 0, 12),
    (2, 32, 32, 64, 32, 12),
    (2, 16, 32, 32, 0, 0),       # 256-pixel windows, 32-channel tile (16-wide rows)
])
def test_conv_fwd_stats_epilogue(cuda_dev, N, H, Cin, Cout, C2, tile):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    x2 = torch.randn(N, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin + C2, Cout, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cout, device=cuda_dev)
    z = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    wp = pack_fwd(w)            # kept alive: the kernel reads it after later allocations
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, C2=C2, src1=ptr(x),
             src2=ptr(x2) if C2 else None, wgt=ptr(wp), bias=ptr(b), Cout=Cout, relu=0, dst1=ptr(z), tile=tile)
    rows, px = C().conv_stat_tiles(dict(d, stats=1))
    assert rows > 0
    st = torch.full((rows, 2, Cout), float("nan"), device=cuda_dev)
    C().conv_fwd(dict(d, stats=ptr(st)), stream())
    torch.cuda.synchronize()
    xin = torch.cat([nchw(x.float()), nchw(x2.float())], 1) if C2 else nchw(x.float())
    ref = nhwc(F.conv2d(xin, w.float().permute(3, 2, 0, 1), b, padding=1))
    assert rel_err(z, ref) < 1e-2
    assert torch.isfinite(st).all()
    mom = _moments(z)
    tot = st.sum(0)
    assert torch.allclose(tot, mom.sum(0), rtol=1e-4, atol=1e-2 * H), (tot - mom.sum(0)).abs().max()
    if (H * H) % px == 0 and rows % N == 0:
        per = st.view(N, rows // N, 2, Cout).sum(1)
        assert torch.allclose(per, mom, rtol=1e-4, atol=1e-2 * H)


def _keep(q_idx, C, seed, salt, rate):
    from unet_distributed_amd.models.reference import _hash_u32
    h = _hash_u32(q_idx, seed, salt)
    return h >= int(rate * 4294967296.0)


@pytest.mark.parametrize("N,H,Cg,Cy,gn,drop,tile", [
    (2, 64, 64, 32, False, 0.0, 0),     # row window dgrad (d: 64 -> 32 channels), BatchNorm coefficients
    (2, 32, 64, 64, True, 0.2, 0),      # GroupNorm coefficients + dropout keep recomputed
    (8, 8, 256, 128, False, 0.2, 0),    # implicit GEMM dgrad (8-wide)
    (4, 16, 128, 64, True, 0.0, 0),     # 16-wide window, GroupNorm
    (2, 32, 64, 64, True, 0.2, 12),     # 64-channel row window
    (2, 128, 32, 64, False, 0.0, 12),
])
def test_conv_dgrad_norm_epilogue(cuda_dev, N, H, Cg, Cy, gn, drop, tile):
    """dgrad of a conv whose input y = dropout(relu(a z + c)): g = dgrad * mask, stats."""
    torch.manual_seed(1)
    dz = torch.randn(N, H, H, Cg, device=cuda_dev).bfloat16()       # gradient at the conv's output
    w = (torch.randn(3, 3, Cy, Cg, device=cuda_dev) * 0.1).bfloat16()
    z = torch.randn(N, H, H, Cy, device=cuda_dev).bfloat16()         # pre-norm input of the conv
    rows_c = N if gn else 1
    a = (0.5 + torch.rand(rows_c, Cy, device=cuda_dev))
    c = 0.3 * torch.randn(rows_c, Cy, device=cuda_dev)
    g = torch.empty(N, H, H, Cy, device=cuda_dev, dtype=torch.bfloat16)
    seed, salt = 1234, 7
    wp = pack_dgrad(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cg, src1=ptr(dz), wgt=ptr(wp),
             Cout=Cy, relu=0, dst1=ptr(g), nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=Cy if gn else 0,
             npix=H * H, nd_rate=drop, nd_salt=salt, seed=seed, tile=tile)
    rows, px = C().conv_stat_tiles(dict(d, stats=1))
    assert rows > 0
    st = torch.full((rows, 2, Cy), float("nan"), device=cuda_dev)
    C().conv_fwd(dict(d, stats=ptr(st)), stream())
    torch.cuda.synchronize()
    xr = torch.zeros(N, Cy, H, H, device=cuda_dev, requires_grad=True)
    (gref,) = torch.autograd.grad(F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1), xr, nchw(dz.float()))
    gref = nhwc(gref)
    ai = a.view(rows_c, 1, 1, Cy) if gn else a.view(1, 1, 1, Cy)
    ci = c.view(rows_c, 1, 1, Cy) if gn else c.view(1, 1, 1, Cy)
    mask = (ai * z.float() + ci) > 0
    scale = 1.0
    if drop > 0:
        q = torch.arange(N * H * H * Cy, device=cuda_dev, dtype=torch.int64).view(N, H, H, Cy)
        mask = mask & _keep(q, Cy, seed, salt, drop)
        scale = 1.0 / (1.0 - drop)
    gref = gref * mask * scale
    assert rel_err(g, gref) < 1e-2
    gf, zf = g.float().reshape(N, -1, Cy), z.float().reshape(N, -1, Cy)
    mom = torch.stack([gf.sum(1), (gf * zf).sum(1)], 1)
    tot = st.sum(0)
    assert torch.allclose(tot, mom.sum(0), rtol=1e-3, atol=1e-2 * H)
    if (H * H) % px == 0 and rows % N == 0:
        per = st.view(N, rows // N, 2, Cy).sum(1)
        assert torch.allclose(per, mom, rtol=1e-3, atol=1e-2 * H)


@pytest.mark.parametrize("N,H,Cg,Cy,gn,tile", [
    (2, 128, 32, 32, False, 0),     # level-1 shape (128-wide rows), BatchNorm coefficients
    (2, 64, 64, 64, True, 0),       # GroupNorm coefficients
    (4, 16, 256, 256, False, 0),    # 16-wide rows
    (2, 32, 128, 128, True, 12),    # 64-channel row window
])
def test_dgrad_norm_skip_half_with_fused_pool_backward(cuda_dev, N, H, Cg, Cy, gn, tile):
    """Skip half of a decoder data gradient into a normalised convNb output y =
    relu(a z + c) that was also max-pooled: the epilogue adds the pooled gradient at
    each window's argmax (route_gy), masks by the recomputed ReLU and writes the
    {sum g, sum g z} rows -- the dskip tensor + pool_bwd_norm pass it replaces."""
    torch.manual_seed(11)
    dz = torch.randn(N, H, H, Cg, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cy, Cg, device=cuda_dev) * 0.1).bfloat16()
    z = torch.randn(N, H, H, Cy, device=cuda_dev).bfloat16()
    rows_c = N if gn else 1
    a = 0.5 + torch.rand(rows_c, Cy, device=cuda_dev)
    c = 0.3 * torch.randn(rows_c, Cy, device=cuda_dev)
    ai = a.view(rows_c, 1, 1, Cy) if gn else a.view(1, 1, 1, Cy)
    ci = c.view(rows_c, 1, 1, Cy) if gn else c.view(1, 1, 1, Cy)
    y = torch.relu(ai * z.float() + ci).bfloat16()
    pooled = torch.empty(N, H // 2, H // 2, Cy, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * Cy // 8, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, Cy, 0], [], stream())
    dpool = torch.randn(N, H // 2, H // 2, Cy, device=cuda_dev).bfloat16()
    routed = torch.empty_like(y)
    C().generic("pool_bwd", [0, ptr(dpool), 0, ptr(routed), ptr(codes)], [N, 1, H, H, Cy, 0], [], stream())
    g = torch.empty_like(y)
    wp = pack_dgrad(w)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cg, src1=ptr(dz), wgt=ptr(wp),
             Cout=Cy, relu=0, dst1=ptr(g), nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=Cy if gn else 0,
             npix=H * H, route_gy=ptr(dpool), pool_code=ptr(codes), tile=tile)
    rows, px = C().conv_stat_tiles(dict(d, stats=1))
    assert rows > 0
    st = torch.full((rows, 2, Cy), float("nan"), device=cuda_dev)
    C().conv_fwd(dict(d, stats=ptr(st)), stream())
    torch.cuda.synchronize()
    xr = torch.zeros(N, Cy, H, H, device=cuda_dev, requires_grad=True)
    (gref,) = torch.autograd.grad(F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1), xr, nchw(dz.float()))
    gref = (nhwc(gref) + routed.float()) * ((ai * z.float() + ci) > 0)
    assert routed.float().abs().sum() > 0
    assert rel_err(g, gref) < 1e-2
    gf, zf = g.float().reshape(N, -1, Cy), z.float().reshape(N, -1, Cy)
    mom = torch.stack([gf.sum(1), (gf * zf).sum(1)], 1)
    assert torch.allclose(st.sum(0), mom.sum(0), rtol=1e-3, atol=1e-2 * H)
    if (H * H) % px == 0 and rows % N == 0:
        per = st.view(N, rows // N, 2, Cy).sum(1)
        assert torch.allclose(per, mom, rtol=1e-3, atol=1e-2 * H)


def test_tconv_dgrad_norm_epilogue(cuda_dev):
    """2x2 stride-2 transposed-conv data gradient (window kernel, 32-wide coarse rows)
    writing the gradient of a BatchNorm'd activation."""
    torch.manual_seed(2)
    N, Hc, Ci, Co = 2, 32, 64, 32        # coarse Hc x Hc x Ci -> fine 2Hc x 2Hc x Co
    dout = torch.randn(N, 2 * Hc, 2 * Hc, Co, device=cuda_dev).bfloat16()
    wk = (torch.randn(2, 2, Co, Ci, device=cuda_dev) * 0.1).bfloat16()      # (kh, kw, Cout, Cin)
    z = torch.randn(N, Hc, Hc, Ci, device=cuda_dev).bfloat16()
    a = 0.5 + torch.rand(Ci, device=cuda_dev)
    c = 0.3 * torch.randn(Ci, device=cuda_dev)
    g = torch.empty(N, Hc, Hc, Ci, device=cuda_dev, dtype=torch.bfloat16)
    # dgrad weights: [Ci][tap (kh, kw)][Co]
    wdg = torch.zeros(Ci, 64 * ((4 * Co + 63) // 64), device=cuda_dev, dtype=torch.bfloat16)
    wdg[:, :4 * Co] = wk.permute(3, 0, 1, 2).reshape(Ci, 4 * Co)
    d = dict(N=N, OH=Hc, OW=Hc, IH=2 * Hc, IW=2 * Hc, KH=2, KW=2, stride=2, pad=0, C1=Co, src1=ptr(dout),
             wgt=ptr(wdg), Cout=Ci, relu=0, dst1=ptr(g), nz=ptr(z), na=ptr(a), nc=ptr(c), ncs=0, npix=Hc * Hc)
    rows, px = C().conv_stat_tiles(dict(d, stats=1))
    assert rows > 0 and px == 256
    st = torch.zeros(rows, 2, Ci, device=cuda_dev)
    C().conv_fwd(dict(d, stats=ptr(st)), stream())
    torch.cuda.synchronize()
    xr = torch.zeros(N, Ci, Hc, Hc, device=cuda_dev, requires_grad=True)
    (gref,) = torch.autograd.grad(F.conv_transpose2d(xr, wk.float().permute(3, 2, 0, 1), stride=2), xr,
                                  nchw(dout.float()))
    gref = nhwc(gref) * ((a * z.float() + c) > 0)
    assert rel_err(g, gref) < 1e-2
    gf, zf = g.float().reshape(-1, Ci), z.float().reshape(-1, Ci)
    assert torch.allclose(st.sum(0), torch.stack([gf.sum(0), (gf * zf).sum(0)]), rtol=1e-3, atol=0.5)


def test_maxpool_all_zero_window_routes_nothing(cuda_dev):
    """A 2x2 window of clipped (zero) ReLU outputs passes no gradient (relu'(0) = 0);
    the argmax-code and recompute paths agree."""
    N, H, Cc = 1, 4, 8
    x = torch.zeros(N, H, H, Cc, device=cuda_dev, dtype=torch.bfloat16)
    x[0, 0, 0, :] = 1.0                  # window (0, 0) has a positive max, the others are all zero
    y = torch.empty(N, H // 2, H // 2, Cc, device=cuda_dev, dtype=torch.bfloat16)
    code = torch.zeros(y.numel() // 8, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(x), ptr(y), ptr(code)], [N, 1, H, H, Cc, 0], [], stream())
    dy = torch.ones_like(y)
    dx1, dx2 = torch.empty_like(x), torch.empty_like(x)
    C().generic("pool_bwd", [ptr(x), ptr(dy), 0, ptr(dx1)], [N, 1, H, H, Cc, 0], [], stream())
    C().generic("pool_bwd", [0, ptr(dy), 0, ptr(dx2), ptr(code)], [N, 1, H, H, Cc, 0], [], stream())
    torch.cuda.synchronize()
    ref = torch.zeros_like(x)
    ref[0, 0, 0, :] = 1.0
    assert torch.equal(dx1, ref) and torch.equal(dx2, ref)


@pytest.mark.parametrize("N,H,Cc,dims3", [(4, 32, 32, 0), (2, 16, 64, 0), (2, 8, 32, 1)])
def test_pool_bwd_norm_rows(cuda_dev, N, H, Cc, dims3):
    """pool_bwd_norm writes the same gradient as the code-driven pool backward and
    per-sample rows summing to {sum g, sum g z}."""
    torch.manual_seed(4)
    D = 4 if dims3 else 1
    shape = (N, D, H, H, Cc) if dims3 else (N, H, H, Cc)
    x = F.relu(torch.randn(*shape, device=cuda_dev)).bfloat16()
    z = torch.randn(*shape, device=cuda_dev).bfloat16()
    oshape = (N, D // 2, H // 2, H // 2, Cc) if dims3 else (N, H // 2, H // 2, Cc)
    y = torch.empty(*oshape, device=cuda_dev, dtype=torch.bfloat16)
    code = torch.zeros(y.numel() // 8, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(x), ptr(y), ptr(code)], [N, D, H, H, Cc, dims3], [], stream())
    dy = torch.randn_like(y.float()).bfloat16()
    skip = torch.randn_like(x.float()).bfloat16()
    dx_ref, dx = torch.empty_like(x), torch.empty_like(x)
    C().generic("pool_bwd", [0, ptr(dy), ptr(skip), ptr(dx_ref), ptr(code)], [N, D, H, H, Cc, dims3], [], stream())
    nbp = 3
    rows = torch.full((N * nbp, 2, Cc), float("nan"), device=cuda_dev)
    C().generic("pool_bwd_norm", [ptr(code), ptr(dy), ptr(skip), ptr(z), ptr(dx), ptr(rows)],
                [N, D, H, H, Cc, dims3, nbp], [], stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    gf, zf = dx.float().reshape(N, -1, Cc), z.float().reshape(N, -1, Cc)
    mom = torch.stack([gf.sum(1), (gf * zf).sum(1)], 1)
    per = rows.view(N, nbp, 2, Cc).sum(1)
    assert torch.allclose(per, mom, rtol=1e-4, atol=1e-2)


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("N,H,Cin,Cout,gn,tile,stats", [
    (2, 128, 32, 32, False, 6, True),       # 512-pixel windows, BatchNorm coefficients, stats epilogue
    (2, 64, 64, 64, True, 0, True),         # 64-channel tile, GroupNorm (per-sample) coefficients
    (4, 16, 128, 128, False, 0, True),      # 16-wide rows, 4 K chunks
    (2, 128, 32, 32, True, 6, False),       # eval-style generic epilogue
    (4, 16, 32, 32, True, 0, False),        # 256-pixel windows, 32-channel tile (16-wide rows)
])
def test_conv_fwd_operand_norm_on_load(cuda_dev, N, H, Cin, Cout, gn, tile, stats):
    """xform 1: the conv reads the PRE-norm z of its input and normalises it in LDS
    (relu(a z + b)); equals the conv of the materialised activation, and xout holds
    that activation (written once per pixel)."""
    torch.manual_seed(50)
    z = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    rows = N if gn else 1
    a = 0.5 + torch.rand(rows, Cin, device=cuda_dev)
    b = 0.3 * torch.randn(rows, Cin, device=cuda_dev)
    ai = a.view(rows, 1, 1, Cin)
    bi = b.view(rows, 1, 1, Cin)
    y_ref = _bf(torch.clamp(ai.double() * z.double() + bi.double(), min=0).float())
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.1).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    out = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    yo = torch.full_like(z, float("nan"))
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(z), wgt=ptr(wp), bias=ptr(bias),
             Cout=Cout, relu=0, dst1=ptr(out), tile=tile, xform=1, xa=ptr(a), xb=ptr(b), xcs=Cin if gn else 0,
             xout=ptr(yo))
    st = None
    if stats:
        nr, _ = C().conv_stat_tiles(dict(d, stats=1))
        st = torch.zeros(nr, 2, Cout, device=cuda_dev)
        d["stats"] = ptr(st)
    C().conv_fwd(d, stream())
    torch.cuda.synchronize()
    ref = nhwc(F.conv2d(nchw(y_ref.float()), w.float().permute(3, 2, 0, 1), bias, padding=1))
    assert rel_err(out, ref) < 1e-2
    assert torch.isfinite(yo.float()).all()
    assert (yo.float() - y_ref.float()).abs().max() <= 1e-2 * y_ref.float().abs().max()
    if stats:
        tot = st.sum(0)
        zf = out.float().reshape(-1, Cout)
        assert torch.allclose(tot[0], zf.sum(0), rtol=1e-3, atol=1e-2 * H)


@pytest.mark.parametrize("N,H,Ch,gn,dims3", [(2, 64, 32, False, 0), (3, 32, 64, True, 0), (2, 16, 32, True, 1)])
def test_norm_pool_matches_apply_then_pool(cuda_dev, N, H, Ch, gn, dims3):
    """norm_pool (normalise a convNb output and max-pool it in one pass) writes the
    activation, the pooled tensor and the argmax codes of norm_apply + pool_fwd."""
    torch.manual_seed(52)
    D = H if dims3 else 1
    shape = (N, D, H, H, Ch) if dims3 else (N, H, H, Ch)
    z = torch.randn(*shape, device=cuda_dev).bfloat16()
    rows = N if gn else 1
    fa = 0.5 + torch.rand(rows, Ch, device=cuda_dev)
    fc = 0.3 * torch.randn(rows, Ch, device=cuda_dev)
    view = (rows,) + (1,) * (len(shape) - 2) + (Ch,)
    y_ref = torch.clamp(fa.view(view).double() * z.double() + fc.view(view).double(), min=0).float().bfloat16()
    y = torch.empty_like(z)
    pshape = (N, D // 2, H // 2, H // 2, Ch) if dims3 else (N, H // 2, H // 2, Ch)
    py, py_ref = torch.empty(pshape, device=cuda_dev, dtype=torch.bfloat16), torch.empty(pshape, device=cuda_dev,
                                                                                         dtype=torch.bfloat16)
    n_codes = py.numel() // 8
    code, code_ref = [torch.zeros(n_codes, device=cuda_dev, dtype=torch.int32) for _ in range(2)]
    C().generic("norm_pool", [ptr(z), ptr(fa), ptr(fc), ptr(y), ptr(py), ptr(code)],
                [N, D, H, H, Ch, dims3, Ch if gn else 0], [], stream())
    C().generic("pool_fwd", [ptr(y_ref), ptr(py_ref), ptr(code_ref)], [N, D, H, H, Ch, dims3], [], stream())
    torch.cuda.synchronize()
    assert (y.float() - y_ref.float()).abs().max() <= 1e-2 * y_ref.float().abs().max()
    same = torch.equal(y, y_ref)
    if same:        # identical activations -> identical pool outputs and codes
        assert torch.equal(py, py_ref) and torch.equal(code, code_ref)
    else:
        assert (py.float() - py_ref.float()).abs().max() <= 1e-2 * py_ref.float().abs().max()


@pytest.mark.parametrize("N,H,Ch,gn", [(2, 64, 32, False), (3, 32, 32, True), (2, 32, 64, True), (2, 16, 16, False)])
def test_norm_head_logits(cuda_dev, N, H, Ch, gn):
    """norm_head: the head input's activation y = relu(fa z + fc) and the 1x1 head
    logits sum_c y w + b in one pass."""
    torch.manual_seed(53)
    z = torch.randn(N, H, H, Ch, device=cuda_dev).bfloat16()
    rows = N if gn else 1
    fa = 0.5 + torch.rand(rows, Ch, device=cuda_dev)
    fc = 0.3 * torch.randn(rows, Ch, device=cuda_dev)
    w = 0.2 * torch.randn(Ch, device=cuda_dev)
    b = 0.1 * torch.randn(1, device=cuda_dev)
    y_ref = torch.clamp(fa.view(rows, 1, 1, Ch).double() * z.double() + fc.view(rows, 1, 1, Ch).double(),
                        min=0).float().bfloat16()
    y = torch.empty_like(z)
    logit = torch.zeros(N * H * H, device=cuda_dev)
    C().generic("norm_head", [ptr(z), ptr(fa), ptr(fc), ptr(w), ptr(b), ptr(y), ptr(logit)],
                [N * H * H, Ch, Ch if gn else 0, H * H], [], stream())
    torch.cuda.synchronize()
    assert (y.float() - y_ref.float()).abs().max() <= 1e-2 * y_ref.float().abs().max()
    ref = (y.float().reshape(-1, Ch) * w).sum(1) + b
    assert torch.allclose(logit, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("N,H,Ch,gn", [(2, 64, 32, False), (3, 32, 32, True), (2, 32, 64, True), (4, 16, 16, False)])
def test_norm_head_loss_and_backward(cuda_dev, N, H, Ch, gn):
    """norm_head_loss -> head_norm_coef -> head_norm_bwd (the norm-mode training head,
    head.hip) against an fp32 autograd-free reference: probabilities and loss sums, the
    1x1 head's weight / bias gradient (of the unrounded activation relu(fa z + fc),
    formed from the masked z sums), the head input's norm-backward rows {sum g, sum g z}
    of g = dlogit w [fa z + fc > 0] (per sample), and dz = ca g + cb z + cc."""
    torch.manual_seed(54)
    P = H * H
    z = torch.randn(N, H, H, Ch, device=cuda_dev).bfloat16()
    rows_c = N if gn else 1
    fa = 0.5 + torch.rand(rows_c, Ch, device=cuda_dev)
    fc = 0.3 * torch.randn(rows_c, Ch, device=cuda_dev)
    w = 0.2 * torch.randn(Ch, device=cuda_dev)
    b = 0.1 * torch.randn(1, device=cuda_dev)
    t = (torch.rand(N, H, H, device=cuda_dev) > 0.7).to(torch.bfloat16)
    nparts = C().hn_partial_floats(N, P, Ch)
    part = torch.full((nparts,), float("nan"), device=cuda_dev)
    prob = torch.zeros(N * P, device=cuda_dev)
    sums = torch.zeros(4, device=cuda_dev)
    cs = Ch if gn else 0
    C().generic("norm_head_loss", [ptr(z), ptr(fa), ptr(fc), ptr(w), ptr(b), ptr(t), 0, ptr(prob), ptr(part),
                                   ptr(sums)], [N, P, Ch, cs], [], stream())
    torch.cuda.synchronize()
    # fp64 product + sum rounds like the kernel's fmaf (the 16-bit y then matches)
    v = (fa.view(rows_c, 1, Ch).double() * z.double().view(N, P, Ch) + fc.view(rows_c, 1, Ch).double()).float()
    y = torch.clamp(v, min=0).bfloat16().float()
    logit = (y * w).sum(-1) + b                                  # [N, P]
    pr = torch.sigmoid(logit)
    tf = t.float().view(N, P)
    assert torch.allclose(prob.view(N, P), pr, rtol=1e-3, atol=1e-4)
    bce = torch.clamp(logit, min=0) - logit * tf + torch.log1p(torch.exp(-logit.abs()))
    ref_sums = torch.stack([(tf * pr).sum(), tf.sum(), pr.sum(), bce.sum()])
    assert torch.allclose(sums, ref_sums, rtol=1e-4, atol=1e-2)
    # backward from the forward's sums
    inv_total, bce_w, gs = 1.0 / (N * P), 0.3, 2.0
    nbp = C().hn_blocks_per_sample(N, P)
    rows = torch.full((N * nbp, 2, Ch), float("nan"), device=cuda_dev)
    gw, gb = torch.zeros(Ch, device=cuda_dev), torch.zeros(1, device=cuda_dev)
    C().generic("head_norm_coef", [ptr(part), ptr(sums), ptr(w), ptr(fa), ptr(fc), ptr(rows), ptr(gw), ptr(gb)],
                [N, P, Ch, cs], [inv_total, bce_w, gs], stream())
    ca = 0.5 + torch.rand(rows_c, Ch, device=cuda_dev)
    cb = 0.2 * torch.randn(rows_c, Ch, device=cuda_dev)
    cc = 0.1 * torch.randn(rows_c, Ch, device=cuda_dev)
    dz = torch.full_like(z, float("nan"))
    C().generic("head_norm_bwd", [ptr(z), ptr(prob), ptr(t), ptr(sums), ptr(w), ptr(fa), ptr(fc), ptr(ca), ptr(cb),
                                  ptr(cc), ptr(dz)], [N, P, Ch, cs], [inv_total, bce_w, gs], stream())
    torch.cuda.synchronize()
    I, St, Sp = ref_sums[0], ref_sums[1], ref_sums[2]
    dl = gs * ((-2.0 / (2 * I + 1) * tf + 1.0 / (St + Sp + 1)) * pr * (1 - pr) + bce_w * (pr - tf) * inv_total)
    g = dl.unsqueeze(-1) * w * (v > 0).float()                   # [N, P, C]
    zf = z.float().view(N, P, Ch)
    ref_rows = torch.stack([g.sum(1), (g * zf).sum(1)], 1)       # per sample [N, 2, C]
    got = rows.view(N, nbp, 2, Ch).sum(1)
    scale = ref_rows.abs().max()
    assert (got - ref_rows).abs().max() <= 1e-3 * scale, (got - ref_rows).abs().max()
    ref_gw = (dl.unsqueeze(-1) * torch.clamp(v, min=0)).sum((0, 1))      # of the unrounded y
    assert (gw - ref_gw).abs().max() <= 1e-3 * ref_gw.abs().max()
    assert abs(gb.item() - dl.sum().item()) <= 1e-3 * dl.abs().sum().item()
    ref_dz = ca.view(rows_c, 1, Ch) * g + cb.view(rows_c, 1, Ch) * zf + cc.view(rows_c, 1, Ch)
    assert (dz.float().view(N, P, Ch) - ref_dz).abs().max() <= 1e-2 * ref_dz.abs().max()


@pytest.mark.parametrize("N,H,Cpad,gn,splits", [(2, 128, 4, False, 3), (3, 64, 8, True, 5), (4, 32, 4, True, 2)])
def test_first_layer_wgrad_dz_on_load(cuda_dev, N, H, Cpad, gn, splits):
    """First-layer window wgrad with the B transform (WgradParams xform 2): b = g and
    dz = xa g + xb z + xc formed in LDS gives the weight / bias gradient of the
    materialised dz (the norm backward's dz of the first layer is never stored)."""
    from test_gpu_kernels import _wgrad
    torch.manual_seed(56)
    Co = 32
    x = torch.randn(N, H, H, Cpad, device=cuda_dev).bfloat16()
    g = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    z = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    rows = N if gn else 1
    ca = 0.5 + torch.rand(rows, Co, device=cuda_dev)
    cb = 0.2 * torch.randn(rows, Co, device=cuda_dev)
    cc = 0.1 * torch.randn(rows, Co, device=cuda_dev)
    v = lambda t: t.view(rows, 1, 1, Co).double()
    dz = (v(ca) * g.double() + (v(cb) * z.double() + v(cc))).float().bfloat16()
    BM = C().wgrad_pick(Cpad, 0, Co, 9, QW=H, win=0)[0]
    Mtot = (9 * Cpad + BM - 1) // BM * BM
    base = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=Cpad, a1=ptr(x), Nc=Co, bias_mode=1, win=0)
    kw = dict(bias_w=(splits, Co), rows=(Cpad, Cpad))
    g0, b0 = _wgrad(dict(base, b=ptr(dz)), splits, 1, Mtot, 9 * Cpad, Co, 9 * Cpad * Co, **kw)
    g1, b1 = _wgrad(dict(base, b=ptr(g), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z),
                         xcs=Co if gn else 0), splits, 1, Mtot, 9 * Cpad, Co, 9 * Cpad * Co, **kw)
    torch.cuda.synchronize()
    assert rel_err(g1, g0) < 1e-2, rel_err(g1, g0)
    assert rel_err(b1, b0) < 1e-2, rel_err(b1, b0)


def _stats_ref(rows, Ch):
    s = rows.double().reshape(-1, 2, Ch).sum(0)
    return s[0], s[1]


@pytest.mark.parametrize("R,Ch", [(128 * 37 + 5, 32), (20000 + 13, 64), (4096 * 9 + 1, 512), (31, 256)])
def test_bn_stats_single_launch_many_slices(cuda_dev, R, Ch):
    """bn_stats_fused_kernel directly (norm.hip): R rows large enough that the phase-1 grid
    has far more than 32 slices with a ragged last slice (the 8-way unrolled slice loop and
    its tail both run), modes 0 (forward) and 1 (backward), each launched twice on the same
    workspace (the last block must reset the hand-off counter)."""
    g = torch.Generator(device="cuda").manual_seed(R)
    dev = cuda_dev
    rows = torch.randn(R, 2, Ch, device=dev, generator=g)
    rows[:, 1] = rows[:, 1].abs() * 3 + 2          # second moment rows: keep var > 0
    count = float(R * 16)
    eps, mom = 1e-3, 0.01
    gamma = torch.rand(Ch, device=dev, generator=g) + 0.5
    beta = torch.randn(Ch, device=dev, generator=g)
    ws = torch.zeros(C().row_slices(R) * 2 * Ch + 64, device=dev)
    f = lambda: torch.zeros(Ch, device=dev)
    mean, rstd, fa, fc, ca, cb, cc, dg, db = (f() for _ in range(9))
    rm, rv = f(), torch.ones(Ch, device=dev)
    s1, s2 = _stats_ref(rows, Ch)
    mu = s1 / count
    var = (s2 / count - mu * mu).clamp_min(0)
    r = torch.rsqrt(var + eps)
    rm_ref, rv_ref = rm.double().clone(), rv.double().clone()
    for rep in range(2):
        C().generic("bn_stats", [ptr(rows), ptr(gamma), ptr(beta), ptr(rm), ptr(rv), ptr(mean), ptr(rstd), ptr(fa),
                                 ptr(fc), 0, 0, 0, 0, 0, ptr(ws)], [R, Ch, 0], [count, eps, mom], stream())
        torch.cuda.synchronize()
        rm_ref = (1 - mom) * rm_ref + mom * mu
        rv_ref = (1 - mom) * rv_ref + mom * var * (count / (count - 1))
        assert torch.allclose(mean.double(), mu, rtol=1e-5, atol=1e-6), rep
        assert torch.allclose(rstd.double(), r, rtol=1e-4), rep
        assert torch.allclose(fa.double(), gamma.double() * r, rtol=1e-4), rep
        assert torch.allclose(fc.double(), beta.double() - mu * gamma.double() * r, rtol=1e-4, atol=1e-5), rep
        assert torch.allclose(rm.double(), rm_ref, rtol=1e-5, atol=1e-6), rep
        assert torch.allclose(rv.double(), rv_ref, rtol=1e-5, atol=1e-6), rep
        assert ws[-64:].abs().sum().item() == 0, "hand-off counter not reset"
    # backward (mode 1): rows = {sum g, sum g z}; mean / rstd from the forward above
    grows = torch.randn(R, 2, Ch, device=dev, generator=g)
    t1, t2 = _stats_ref(grows, Ch)
    gm, mu_, r_ = gamma.double(), mean.double(), rstd.double()
    sgx = r_ * (t2 - mu_ * t1)
    for rep in range(2):
        C().generic("bn_stats", [ptr(grows), ptr(gamma), ptr(beta), 0, 0, ptr(mean), ptr(rstd), 0, 0, ptr(ca),
                                 ptr(cb), ptr(cc), ptr(dg), ptr(db), ptr(ws)], [R, Ch, 1], [count, eps, mom], stream())
        torch.cuda.synchronize()
        tol = dict(rtol=1e-4, atol=1e-3 * (t1.abs().max().item() + 1) / count + 1e-6)
        assert torch.allclose(db.double(), t1, rtol=1e-5, atol=1e-3), rep
        assert torch.allclose(dg.double(), sgx, rtol=1e-4, atol=1e-3), rep
        assert torch.allclose(ca.double(), gm * r_, rtol=1e-5), rep
        assert torch.allclose(cb.double(), -gm * r_ * r_ * sgx / count, **tol), rep
        assert torch.allclose(cc.double(), -gm * r_ * t1 / count + gm * r_ * r_ * mu_ * sgx / count, **tol), rep
        assert ws[-64:].abs().sum().item() == 0


@pytest.mark.parametrize("N,rps,Ch,G", [(4100, 2, 32, 8), (37, 3, 512, 32)])
def test_gn_stats_backward_parameter_grads_many_samples(cuda_dev, N, rps, Ch, G):
    """gn_stats mode 1: per-sample backward coefficients, and the dgamma / dbeta column sums
    of the per-sample contributions through the single-launch slice reduction (N = 4100
    samples: more than 32 slices, ragged last), launched twice on one workspace."""
    g = torch.Generator(device="cuda").manual_seed(N)
    dev = cuda_dev
    P = 64
    Cg = Ch // G
    mean = torch.randn(N, G, device=dev, generator=g).repeat_interleave(Cg, 1).contiguous()
    rstd = (torch.rand(N, G, device=dev, generator=g) + 0.5).repeat_interleave(Cg, 1).contiguous()
    gamma = torch.rand(Ch, device=dev, generator=g) + 0.5
    beta = torch.zeros(Ch, device=dev)
    rows = torch.randn(N * rps, 2, Ch, device=dev, generator=g)
    S = rows.double().reshape(N, rps, 2, Ch).sum(1)                  # [N, 2, Ch]
    mu, r = mean.double(), rstd.double()
    contrib1 = S[:, 0]
    contrib2 = r * (S[:, 1] - mu * S[:, 0])
    db_ref, dg_ref = contrib1.sum(0), contrib2.sum(0)
    work = torch.zeros(N * 2 * Ch + C().row_slices(N) * 2 * Ch + C().row_slices(N) * 2 * Ch + 64, device=dev)
    f = lambda: torch.zeros(N * Ch, device=dev)
    ca, cb, cc = f(), f(), f()
    dg, db = torch.zeros(Ch, device=dev), torch.zeros(Ch, device=dev)
    for rep in range(2):
        C().generic("gn_stats", [ptr(rows), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd), 0, 0, ptr(ca), ptr(cb),
                                 ptr(cc), ptr(dg), ptr(db), ptr(work)], [N, rps, Ch, G, P, 1], [1e-3], stream())
        torch.cuda.synchronize()
        assert torch.allclose(db.double(), db_ref, rtol=1e-4, atol=1e-2), rep
        assert torch.allclose(dg.double(), dg_ref, rtol=1e-4, atol=1e-2), rep
        assert torch.allclose(ca.double().view(N, Ch), gamma.double() * r, rtol=1e-5), rep


@pytest.mark.parametrize("N,H,Cin,Cout,tile,n0", [(2, 32, 128, 128, 0, 0), (4, 16, 128, 256, 0, 3),
                                                 (2, 64, 64, 64, 0, 0), (2, 128, 32, 32, 6, 1)])
def test_conv_fwd_operand_norm_on_load_with_dropout(cuda_dev, N, H, Cin, Cout, tile, n0):
    """xform 1 with the source layer's inverted dropout (xd_rate / xd_salt / xd_idx0, the
    planner's conv3a / conv4a): xout equals norm_apply's dropout(relu(a z + b)) bit for bit
    (same hash of the whole-batch element index, n0: the chunk's first image), and the conv
    output equals the same window conv of that materialised activation."""
    torch.manual_seed(51 + N + H)
    dev = cuda_dev
    z = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    a = 0.5 + torch.rand(Cin, device=dev)
    b = 0.3 * torch.randn(Cin, device=dev)
    # norm_apply with gamma = a, rstd = 1, beta = b, mean = 0: its A = a, B = b exactly
    one, zero = torch.ones(Cin, device=dev), torch.zeros(Cin, device=dev)
    y_ap = torch.empty_like(z)
    seed, salt, rate = 1234567, 7, 0.3
    C().generic("norm_apply", [ptr(z), ptr(zero), ptr(one), ptr(a), ptr(b), ptr(y_ap)],
                [N, H * H, Cin, 0, 1, salt, seed, n0], [rate], stream())
    w = (torch.randn(3, 3, Cin, Cout, device=dev) * 0.05).bfloat16()
    bias = torch.randn(Cout, device=dev) * 0.1
    wp = pack_fwd(w)
    base = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, wgt=ptr(wp), bias=ptr(bias), Cout=Cout,
                relu=0, tile=tile)           # (the normalised consumer's pre-norm output, generic epilogue)
    ref = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(base, src1=ptr(y_ap), dst1=ptr(ref)), stream())
    out = torch.empty_like(ref)
    yo = torch.full_like(z, float("nan"))
    C().conv_fwd(dict(base, src1=ptr(z), dst1=ptr(out), xform=1, xa=ptr(a), xb=ptr(b), xcs=0, xout=ptr(yo),
                      xd_rate=rate, xd_salt=salt, xd_idx0=n0 * H * H * Cin, seed=seed), stream())
    torch.cuda.synchronize()
    assert torch.equal(yo, y_ap)
    assert torch.equal(out, ref)
    kept = (y_ap.float() != 0).float().mean().item()
    assert 0.2 < kept < 0.5, kept                      # (about (1 - rate) of the positive half)
