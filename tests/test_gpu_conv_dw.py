"""Fused data + weight gradient (conv_dw.hip): one staged dY halo feeds both.  The data
gradient must equal the split row-window data gradient bit for bit (same operands, same
MFMA order), the slab rows must sum to the fp32 weight / bias gradient of the conv."""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, nchw, nhwc, pack_dgrad, ptr, rel_err, stream

pytestmark = pytest.mark.gpu


def _ref_wgrad(x, dy, w):
    wr = w.float().permute(3, 2, 0, 1).clone().requires_grad_(True)
    xr = nchw(x.float())
    y = F.conv2d(xr, wr, padding=1)
    (gw,) = torch.autograd.grad(y, wr, nchw(dy.float()))
    return gw.permute(2, 3, 1, 0)            # -> [kh][kw][ci][co]


@pytest.mark.parametrize("N,nsplit,mask", [(2, 7, "act"), (3, 64, "bits"), (1, 1, "none"), (4, 512, "bits")])
def test_fused_dgrad_wgrad_matches_split_kernels(cuda_dev, N, nsplit, mask):
    torch.manual_seed(N * 100 + nsplit)
    H = W = 128
    dev = cuda_dev
    dy = torch.randn(N, H, W, 32, device=dev).bfloat16()
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()          # the conv's forward input
    act = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()        # ReLU output the gradient is masked by
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)                       # (kept alive: the launches below read it)
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dy), wgt=ptr(wp),
                Cout=32, relu=0)
    bits = None
    if mask == "act":
        base.update(mask1=ptr(act))
    elif mask == "bits":
        v = (act.float() > 0).reshape(-1, 8).to(torch.int32)
        bits = (v << torch.arange(8, device=dev, dtype=torch.int32)).sum(1).to(torch.uint8)
        base.update(mask1=ptr(bits), mask_bits=1)
    ref_dx = torch.empty(N, H, W, 32, device=dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(base, dst1=ptr(ref_dx)), stream())
    dx = torch.full_like(ref_dx, 7.0)
    slab = torch.full((nsplit + 3, 9, 32, 32), float("nan"), device=dev)
    bslab = torch.full((nsplit + 3, 32), float("nan"), device=dev)
    d = dict(base, dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32,
             fw_nsplit=nsplit, fw_split_lo=3)
    assert C().conv_fwd_grid(d) == nsplit
    C().conv_fwd(d, stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)
    assert torch.isnan(slab[:3]).all() and torch.isnan(bslab[:3]).all()      # rows below split_lo untouched
    gw = slab[3:].double().sum(0).float()                                     # [tap][ci][co]
    ref_w = _ref_wgrad(x, dy, w).reshape(9, 32, 32)
    assert rel_err(gw, ref_w) < 1e-4, rel_err(gw, ref_w)
    gb = bslab[3:].double().sum(0).float()
    assert rel_err(gb, dy.float().sum((0, 1, 2))) < 1e-4


def test_fused_dgrad_wgrad_with_pool_route(cuda_dev):
    """The skip half of a decoder data gradient with the max-pool backward in its epilogue
    (route_gy + codes), as the planner uses it for conv9a."""
    torch.manual_seed(5)
    N, H, W = 2, 128, 128
    dev = cuda_dev
    dy = torch.randn(N, H, W, 32, device=dev).bfloat16()
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    pooled = torch.empty(N, H // 2, W // 2, 32, device=dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) * (W // 2) * 4, device=dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(x), ptr(pooled), ptr(codes)], [N, 1, H, W, 32, 0], [], stream())
    gy = torch.randn(N, H // 2, W // 2, 32, device=dev).bfloat16()
    wp = pack_dgrad(w)
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dy), wgt=ptr(wp),
                Cout=32, relu=0, mask1=ptr(x), route_gy=ptr(gy), pool_code=ptr(codes))
    ref_dx = torch.empty(N, H, W, 32, device=dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(base, dst1=ptr(ref_dx)), stream())
    dx = torch.empty_like(ref_dx)
    slab = torch.zeros(16, 9, 32, 32, device=dev)
    bslab = torch.zeros(16, 32, device=dev)
    C().conv_fwd(dict(base, dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32,
                      fw_nsplit=16), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)
    assert rel_err(slab.double().sum(0).float(), _ref_wgrad(x, dy, w).reshape(9, 32, 32)) < 1e-4


def _norm_bwd_apply(g, z, ca, cb, cc, gn):
    """dz through the split path's own kernel (norm.hip::norm_bwd_apply)."""
    N, H, W, Ch = g.shape
    dz = torch.empty_like(g)
    C().generic("norm_bwd_apply", [ptr(g), ptr(z), ptr(ca), ptr(cb), ptr(cc), ptr(dz)],
                [N, H * W, Ch, Ch if gn else 0], [], stream())
    return dz


@pytest.mark.parametrize("N,nsplit,gn", [(2, 7, False), (3, 64, True), (1, 1, True), (4, 512, False)])
def test_fused_dgrad_wgrad_norm_backward_on_load(cuda_dev, N, nsplit, gn):
    """XF 2: the halo is dz = ca g + cb z + cc formed from g and z in LDS -- the data
    gradient and the slab rows must equal the fused kernel fed the materialised dz
    (norm_bwd_apply) bit for bit, and the weight gradient the fp32 reference."""
    torch.manual_seed(N * 7 + nsplit)
    H = W = 128
    dev = cuda_dev
    g = torch.randn(N, H, W, 32, device=dev).bfloat16()
    z = torch.randn(N, H, W, 32, device=dev).bfloat16()
    rows = N if gn else 1
    ca = 0.5 + torch.rand(rows, 32, device=dev)
    cb = 0.2 * torch.randn(rows, 32, device=dev)
    cc = 0.1 * torch.randn(rows, 32, device=dev)
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    act = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)
    dz = _norm_bwd_apply(g, z, ca, cb, cc, gn)
    outs = []
    for xf in (False, True):
        dx = torch.full((N, H, W, 32), 7.0, device=dev, dtype=torch.bfloat16)
        slab = torch.full((nsplit, 9, 32, 32), float("nan"), device=dev)
        bslab = torch.full((nsplit, 32), float("nan"), device=dev)
        d = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dz), wgt=ptr(wp), Cout=32,
                 relu=0, mask1=ptr(act), dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab),
                 fw_Cx=32, fw_nsplit=nsplit)
        if xf:
            d.update(src1=ptr(g), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z), xcs=32 if gn else 0)
        assert C().conv_fwd_grid(d) == nsplit
        C().conv_fwd(d, stream())
        outs.append((dx, slab, bslab))
    torch.cuda.synchronize()
    (dx0, s0, b0), (dx1, s1, b1) = outs
    assert torch.equal(dx1, dx0)
    assert torch.equal(s1, s0) and torch.equal(b1, b0)
    ref_w = _ref_wgrad(x, dz, w).reshape(9, 32, 32)
    assert rel_err(s1.double().sum(0).float(), ref_w) < 1e-4
    assert rel_err(b1.double().sum(0).float(), dz.float().sum((0, 1, 2))) < 1e-4


@pytest.mark.parametrize("N,gn,xf", [(2, False, False), (3, True, True), (2, False, True)])
def test_fused_dgrad_wgrad_dgrad_norm_epilogue(cuda_dev, N, gn, xf):
    """EPI_DGRAD_NORM in the fused kernel (the destination is itself a normalised
    activation's gradient): dX equals the split row-window dgrad's (same epilogue), the
    per-window {sum g, sum g z} rows sum to the split kernel's per-sample statistics."""
    torch.manual_seed(31 + N)
    H = W = 128
    dev = cuda_dev
    rows = N if gn else 1
    dy = torch.randn(N, H, W, 32, device=dev).bfloat16()
    z = torch.randn(N, H, W, 32, device=dev).bfloat16()
    ca = 0.5 + torch.rand(rows, 32, device=dev)
    cb = 0.2 * torch.randn(rows, 32, device=dev)
    cc = 0.1 * torch.randn(rows, 32, device=dev)
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    zd = torch.randn(N, H, W, 32, device=dev).bfloat16()            # pre-norm z of the destination
    na = 0.5 + torch.rand(rows, 32, device=dev)
    nc = 0.3 * torch.randn(rows, 32, device=dev)
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)
    src = _norm_bwd_apply(dy, z, ca, cb, cc, gn) if xf else dy
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(src), wgt=ptr(wp), Cout=32,
                relu=0, nz=ptr(zd), na=ptr(na), nc=ptr(nc), ncs=32 if gn else 0, npix=H * W)
    g0 = torch.empty(N, H, W, 32, device=dev, dtype=torch.bfloat16)
    r0, _ = C().conv_stat_tiles(dict(base, stats=1, dst1=ptr(g0)))
    st0 = torch.full((r0, 2, 32), float("nan"), device=dev)
    C().conv_fwd(dict(base, dst1=ptr(g0), stats=ptr(st0)), stream())
    slab = torch.zeros(64, 9, 32, 32, device=dev)
    bslab = torch.zeros(64, 32, device=dev)
    fd = dict(base, fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32, fw_nsplit=64)
    if xf:
        fd.update(src1=ptr(dy), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z), xcs=32 if gn else 0)
    r1, px = C().conv_stat_tiles(dict(fd, stats=1, dst1=ptr(g0)))
    assert r1 == N * H // 2 and px == 256
    st1 = torch.full((r1, 2, 32), float("nan"), device=dev)
    g1 = torch.empty_like(g0)
    C().conv_fwd(dict(fd, dst1=ptr(g1), stats=ptr(st1)), stream())
    torch.cuda.synchronize()
    assert torch.equal(g1, g0)
    per0 = st0.double().view(N, -1, 2, 32).sum(1)
    per1 = st1.double().view(N, -1, 2, 32).sum(1)
    assert (per1 - per0).abs().max() <= 1e-4 * per0.abs().max()
    assert rel_err(slab.double().sum(0).float(), _ref_wgrad(x, src, w).reshape(9, 32, 32)) < 1e-4


@pytest.mark.parametrize("N,gn,bce", [(2, False, 0.0), (3, True, 0.5)])
def test_fused_dgrad_wgrad_normalised_head_on_load(cuda_dev, N, gn, bce):
    """XF 3 (the normalised head input conv9b): the halo's dz = (fa z + fc > 0 ? ca w
    dlogit : 0) + cb z + cc is formed from z, the probability and the target -- the data
    gradient and slab rows equal the fused kernel fed head_norm_bwd's materialised dz."""
    torch.manual_seed(77 + N)
    H = W = 128
    dev = cuda_dev
    P = H * W
    rows = N if gn else 1
    z = torch.randn(N, H, W, 32, device=dev).bfloat16()
    prob = torch.rand(N * P, device=dev) * 0.98 + 0.01
    t = (torch.rand(N * P, device=dev) > 0.7).bfloat16()
    sums = torch.tensor([(prob * t.float()).sum().item(), t.float().sum().item(), prob.sum().item(), 0.0],
                        device=dev)
    hw = 0.3 * torch.randn(32, device=dev)
    fa, fc = 0.5 + torch.rand(rows, 32, device=dev), 0.2 * torch.randn(rows, 32, device=dev)
    ca, cb = 0.5 + torch.rand(rows, 32, device=dev), 0.2 * torch.randn(rows, 32, device=dev)
    cc = 0.1 * torch.randn(rows, 32, device=dev)
    gsc = torch.full((1,), 4.0, device=dev)
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    zd = torch.randn(N, H, W, 32, device=dev).bfloat16()            # the destination's pre-norm z
    na, nc = 0.5 + torch.rand(rows, 32, device=dev), 0.3 * torch.randn(rows, 32, device=dev)
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)
    dz = torch.empty_like(z)
    C().generic("head_norm_bwd", [ptr(z), ptr(prob), ptr(t), ptr(sums), ptr(hw), ptr(fa), ptr(fc), ptr(ca), ptr(cb),
                                  ptr(cc), ptr(dz), ptr(gsc)], [N, P, 32, 32 if gn else 0], [1.0 / (N * P), bce, 1.0],
                stream())
    outs = []
    for xf in (False, True):
        dx = torch.full((N, H, W, 32), 7.0, device=dev, dtype=torch.bfloat16)
        slab = torch.full((32, 9, 32, 32), float("nan"), device=dev)
        bslab = torch.full((32, 32), float("nan"), device=dev)
        st = torch.full((N * H // 2, 2, 32), float("nan"), device=dev)
        d = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dz), wgt=ptr(wp), Cout=32,
                 relu=0, nz=ptr(zd), na=ptr(na), nc=ptr(nc), ncs=32 if gn else 0, npix=P, stats=ptr(st),
                 dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32, fw_nsplit=32)
        if xf:
            d.update(src1=ptr(z), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z), xcs=32 if gn else 0,
                     hg_prob=ptr(prob), hg_t=ptr(t), hg_sums=ptr(sums), hg_w=ptr(hw), hg_gscale=ptr(gsc),
                     hg_inv_total=1.0 / (N * P), hg_bce_w=bce, hg_fa=ptr(fa), hg_fc=ptr(fc))
        assert C().conv_fwd_grid(d) == 32
        C().conv_fwd(d, stream())
        outs.append((dx, slab, bslab, st))
    torch.cuda.synchronize()
    (dx0, s0, b0, t0), (dx1, s1, b1, t1) = outs
    assert torch.equal(dx1, dx0) and torch.equal(t1, t0)
    assert torch.equal(s1, s0) and torch.equal(b1, b0)


@pytest.mark.parametrize("N,nsplit,bce", [(2, 16, 0.0), (3, 96, 0.5)])
def test_fused_dgrad_wgrad_head_on_load(cuda_dev, N, nsplit, bce):
    """XF 4 (the norm-free head input conv9b): dY = dlogit w (y > 0) is formed in the halo
    from the probability, the target and the head input's ReLU bits -- the data gradient
    and slab rows equal the fused kernel fed head_bwd's materialised dY bit for bit."""
    torch.manual_seed(90 + N)
    H = W = 128
    dev = cuda_dev
    P = N * H * W
    y = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()      # the head input (conv9b output)
    v = (y.float() > 0).reshape(-1, 8).to(torch.int32)
    bits = (v << torch.arange(8, device=dev, dtype=torch.int32)).sum(1).to(torch.uint8)
    hw = 0.3 * torch.randn(32, device=dev)
    hb = torch.randn(1, device=dev)
    t = (torch.rand(P, device=dev) > 0.7).bfloat16()
    prob = torch.empty(P, device=dev)
    nb = C().head_blocks(P)
    part = torch.empty(nb * 33 + 4 * nb, device=dev)
    sums = torch.empty(4, device=dev)
    C().generic("head_fwd", [ptr(y), ptr(hw), ptr(hb), ptr(t), ptr(prob), ptr(part), ptr(sums)], [P, 32], [], stream())
    dy = torch.empty_like(y)
    ow, ob = torch.empty(32, device=dev), torch.empty(1, device=dev)
    gsc = torch.full((1,), 2.0, device=dev)
    C().generic("head_bwd", [ptr(y), ptr(hw), ptr(prob), ptr(t), ptr(sums), ptr(dy), ptr(part), ptr(ow), ptr(ob),
                             ptr(gsc)], [P, 32], [1.0 / P, bce, 1.0], stream())
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    act = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)
    outs = []
    for xf in (False, True):
        dx = torch.full((N, H, W, 32), 7.0, device=dev, dtype=torch.bfloat16)
        slab = torch.full((nsplit, 9, 32, 32), float("nan"), device=dev)
        bslab = torch.full((nsplit, 32), float("nan"), device=dev)
        d = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dy), wgt=ptr(wp), Cout=32,
                 relu=0, mask1=ptr(act), dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab),
                 fw_Cx=32, fw_nsplit=nsplit)
        if xf:
            d.update(hg_prob=ptr(prob), hg_t=ptr(t), hg_sums=ptr(sums), hg_w=ptr(hw), hg_bits=ptr(bits),
                     hg_gscale=ptr(gsc), hg_inv_total=1.0 / P, hg_bce_w=bce)
        assert C().conv_fwd_grid(d) == nsplit
        C().conv_fwd(d, stream())
        outs.append((dx, slab, bslab))
    torch.cuda.synchronize()
    (dx0, s0, b0), (dx1, s1, b1) = outs
    assert torch.equal(dx1, dx0)
    assert torch.equal(s1, s0) and torch.equal(b1, b0)
    assert rel_err(s1.double().sum(0).float(), _ref_wgrad(x, dy, w).reshape(9, 32, 32)) < 1e-4


@pytest.mark.parametrize("N,W,nsplit", [(2, 256, 9), (1, 512, 64)])
def test_fused_dgrad_wgrad_segmented_rows(cuda_dev, N, W, nsplit):
    """Rows wider than 128 (the 512^2 model) as 128-pixel segments walked segment-major
    (halo columns -1 / 128 from the neighbour segments, the halo-row carry within a
    segment): dX equals the split row-window data gradient, the slabs the fp32 weight /
    bias gradients."""
    torch.manual_seed(W + N)
    H = 64
    dev = cuda_dev
    dy = torch.randn(N, H, W, 32, device=dev).bfloat16()
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    act = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    w = (torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()
    wp = pack_dgrad(w)
    v = (act.float() > 0).reshape(-1, 8).to(torch.int32)
    bits = (v << torch.arange(8, device=dev, dtype=torch.int32)).sum(1).to(torch.uint8)
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(dy), wgt=ptr(wp), Cout=32, relu=0,
                mask1=ptr(bits), mask_bits=1)
    ref_dx = torch.empty(N, H, W, 32, device=dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(base, dst1=ptr(ref_dx)), stream())
    dx = torch.full_like(ref_dx, 7.0)
    slab = torch.full((nsplit, 9, 32, 32), float("nan"), device=dev)
    bslab = torch.full((nsplit, 32), float("nan"), device=dev)
    d = dict(base, dst1=ptr(dx), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32,
             fw_nsplit=nsplit)
    assert C().conv_fwd_grid(d) == nsplit
    C().conv_fwd(d, stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)
    assert rel_err(slab.double().sum(0).float(), _ref_wgrad(x, dy, w).reshape(9, 32, 32)) < 1e-4
    assert rel_err(bslab.double().sum(0).float(), dy.float().sum((0, 1, 2))) < 1e-4
