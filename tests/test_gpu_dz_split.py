"""Norm backward on load in the split consumers (FUSIONS['dz_split']): the data gradient of a
normalised layer on 16..64-wide rows forms its halo as dz = ca g + cb z + cc (conv_win.h XF 2,
the chunk-pipelined DZ variant on 64-wide rows) and the window weight gradient its B operand
(wgrad_win_kernel DZ).  The data gradient must equal the same launch fed the dz that
norm_bwd_apply materialises, bit for bit; the weight gradient the fp32 reference (and the
materialised-dz launch bit for bit where both take the same 32-channel output block)."""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, _wgrad, nchw, pack_dgrad, ptr, rel_err, stream

pytestmark = pytest.mark.gpu


def _coefs(rows, ch, dev):
    return (0.5 + torch.rand(rows, ch, device=dev), 0.2 * torch.randn(rows, ch, device=dev),
            0.1 * torch.randn(rows, ch, device=dev))


def _norm_bwd_apply(g, z, ca, cb, cc, gn):
    N, H, W, Ch = g.shape
    dz = torch.empty_like(g)
    C().generic("norm_bwd_apply", [ptr(g), ptr(z), ptr(ca), ptr(cb), ptr(cc), ptr(dz)],
                [N, H * W, Ch, Ch if gn else 0], [], stream())
    return dz


# (rows W, layer output channels = dgrad input, layer input channels = dgrad output): the
# chunk-pipelined 64-channel window (64, 64, 64), the 32-channel tile on 64-wide rows
# (conv2a), the one-window kernel at 32 / 16-wide rows
@pytest.mark.parametrize("N,W,Co,Ci,gn,norm_epi", [(2, 64, 64, 64, False, False), (3, 64, 64, 64, True, True),
                                                    (2, 64, 64, 32, False, True), (2, 32, 128, 128, True, False),
                                                    (4, 32, 128, 64, False, True), (5, 16, 256, 256, True, True),
                                                    (3, 16, 256, 128, False, False)])
def test_dgrad_dz_on_load_equals_materialised(cuda_dev, N, W, Co, Ci, gn, norm_epi):
    torch.manual_seed(N * 31 + W + Co + Ci)
    dev = cuda_dev
    H = W
    rows = N if gn else 1
    g = torch.randn(N, H, W, Co, device=dev).bfloat16()
    z = torch.randn(N, H, W, Co, device=dev).bfloat16()
    ca, cb, cc = _coefs(rows, Co, dev)
    w = (torch.randn(3, 3, Ci, Co, device=dev) * 0.05).bfloat16()
    wp = pack_dgrad(w)
    dz = _norm_bwd_apply(g, z, ca, cb, cc, gn)
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=Co, wgt=ptr(wp), Cout=Ci, relu=0)
    keep = []
    if norm_epi:        # the destination is itself a normalised activation's gradient
        zd = torch.randn(N, H, W, Ci, device=dev).bfloat16()
        na, nc, _ = _coefs(rows, Ci, dev)
        keep += [zd, na, nc]
        base.update(nz=ptr(zd), na=ptr(na), nc=ptr(nc), ncs=Ci if gn else 0, npix=H * W)
    else:
        act = F.relu(torch.randn(N, H, W, Ci, device=dev)).bfloat16()
        keep.append(act)
        base.update(mask1=ptr(act))
    outs = []
    for xf in (False, True):
        d = dict(base, src1=ptr(dz))
        if xf:
            d.update(src1=ptr(g), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z), xcs=Co if gn else 0)
        dx = torch.full((N, H, W, Ci), 7.0, device=dev, dtype=torch.bfloat16)
        st = None
        if norm_epi:
            r, _ = C().conv_stat_tiles(dict(d, stats=1, dst1=ptr(dx)))
            st = torch.full((r, 2, Ci), float("nan"), device=dev)
            d.update(stats=ptr(st))
        C().conv_fwd(dict(d, dst1=ptr(dx)), stream())
        outs.append((dx, st))
    torch.cuda.synchronize()
    (dx0, st0), (dx1, st1) = outs
    assert torch.isfinite(dx1.float()).all()
    assert torch.equal(dx1, dx0)
    if norm_epi:
        assert torch.equal(st1, st0)


@pytest.mark.parametrize("N,W,Ci,Co,gn,splits", [(2, 64, 64, 64, False, 5), (3, 64, 32, 64, True, 7),
                                                  (2, 32, 128, 128, True, 3), (4, 16, 256, 256, False, 2),
                                                  (3, 64, 64, 32, True, 4)])
def test_wgrad_dz_on_load(cuda_dev, N, W, Ci, Co, gn, splits):
    """Window weight gradient with B = dz formed on load: fp32 reference (weights + bias);
    with 32 output channels the materialised-dz launch takes the same output block and
    must match bit for bit."""
    torch.manual_seed(N * 13 + W + Ci + Co)
    dev = cuda_dev
    H = W
    rows = N if gn else 1
    x = F.relu(torch.randn(N, H, W, Ci, device=dev)).bfloat16()
    g = torch.randn(N, H, W, Co, device=dev).bfloat16()
    z = torch.randn(N, H, W, Co, device=dev).bfloat16()
    ca, cb, cc = _coefs(rows, Co, dev)
    dz = _norm_bwd_apply(g, z, ca, cb, cc, gn)
    base = dict(N=N, QH=H, QW=W, AH=H, AW=W, KH=3, KW=3, pad=1, M1=Ci, a1=ptr(x), Nc=Co, bias_mode=1)
    xfd = dict(base, b=ptr(g), xform=2, xa=ptr(ca), xb=ptr(cb), xc=ptr(cc), xz=ptr(z), xcs=Co if gn else 0)
    gw, gb = _wgrad(xfd, splits, 9, Ci, Ci, Co, 9 * Ci * Co, bias_w=(splits, Co))
    wr = torch.zeros(Co, Ci, 3, 3, device=dev, requires_grad=True)
    br = torch.zeros(Co, device=dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(nchw(x.float()), wr, br, padding=1), [wr, br], nchw(dz.float()))
    assert rel_err(gw, gwr.permute(2, 3, 1, 0).reshape(-1)) < 1e-3
    assert rel_err(gb, gbr) < 1e-3
    if Co == 32:
        gw0, gb0 = _wgrad(dict(base, b=ptr(dz)), splits, 9, Ci, Ci, Co, 9 * Ci * Co, bias_w=(splits, Co))
        assert torch.equal(gw, gw0) and torch.equal(gb, gb0)
