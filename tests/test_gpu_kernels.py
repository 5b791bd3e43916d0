"""Numerics of the gfx950 HIP kernels against fp32 PyTorch references of the same op.

Inputs are bf16-rounded first so the reference sees exactly what the kernel
reads; tolerances cover fp32-accumulate vs bf16 output rounding.
"""

import math

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


def pad64(m):                   # rows zero-padded to a multiple of 64 (the kernels' K step)
    k = m.shape[1]
    kp = (k + 63) // 64 * 64
    out = torch.zeros(m.shape[0], kp, dtype=m.dtype, device=m.device)
    out[:, :k] = m
    return out


def pack_fwd(w_hwio):          # [kh][kw][ci][co] -> [co][kh*kw*ci (pad 64)]
    kh, kw, ci, co = w_hwio.shape
    return pad64(w_hwio.permute(3, 0, 1, 2).reshape(co, kh * kw * ci))


def pack_dgrad(w_hwio):        # -> [ci][taps flipped][co] (pad 64)
    kh, kw, ci, co = w_hwio.shape
    return pad64(w_hwio.flip(0, 1).permute(2, 0, 1, 3).reshape(ci, kh * kw * co))


@pytest.mark.parametrize("N,H,Cin,Cout", [(2, 16, 32, 32), (2, 8, 64, 128), (1, 32, 32, 64), (4, 8, 128, 256)])
def test_conv3x3_fwd_bias_relu(cuda_dev, N, H, Cin, Cout):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cout, device=cuda_dev)
    out = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    wp = pack_fwd(w)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp),
                      bias=ptr(b), Cout=Cout, relu=1, dst1=ptr(out)), stream())
    ref = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(out, ref) < 1e-2


def test_conv3x3_concat_dual_source(cuda_dev):
    """Implicit-GEMM conv (tile 8: row-window off) reading a 64 + 64 channel concat from
    two sources."""
    torch.manual_seed(1)
    N, H, C1, C2, Co = 2, 16, 64, 64, 64
    a = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    skip = torch.randn(N, H, H, C2, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.05).bfloat16()
    out = torch.empty(N, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(skip), wgt=ptr(pack_fwd(w)), Cout=Co, relu=0, dst1=ptr(out), tile=8), stream())
    ref = nhwc(F.conv2d(torch.cat([nchw(a.float()), nchw(skip.float())], 1), w.float().permute(3, 2, 0, 1), padding=1))
    assert rel_err(out, ref) < 1e-2


def test_conv3x3_concat_32_32(cuda_dev):
    torch.manual_seed(12)
    N, H, C1, C2, Co = 2, 16, 32, 32, 32
    a = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    b = torch.randn(N, H, H, C2, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.05).bfloat16()
    out = torch.empty(N, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(b), wgt=ptr(pack_fwd(w)), Cout=Co, relu=0, dst1=ptr(out)), stream())
    ref = nhwc(F.conv2d(torch.cat([nchw(a.float()), nchw(b.float())], 1), w.float().permute(3, 2, 0, 1), padding=1))
    assert rel_err(out, ref) < 1e-2


def test_conv_dgrad_dual_dest_mask(cuda_dev):
    """dgrad of a concat conv: flipped weights, channel split into two tensors, ReLU mask on the skip half."""
    torch.manual_seed(2)
    N, H, C1, C2, Co = 2, 16, 32, 32, 32
    xin = torch.randn(N, H, H, C1 + C2, device=cuda_dev)
    skip = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.1).bfloat16()
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    d1 = torch.empty(N, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy),
                      wgt=ptr(pack_dgrad(w)), Cout=C1 + C2, D1=C1, dst1=ptr(d1), dst2=ptr(d2),
                      mask2=ptr(skip), mask_scale2=1.25), stream())
    xr = nchw(xin).requires_grad_(True)
    y = F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1)
    (g,) = torch.autograd.grad(y, xr, nchw(dy.float()))
    g = nhwc(g)
    ref1 = g[..., :C1]
    ref2 = g[..., C1:] * (skip.float() > 0) * 1.25
    assert rel_err(d1, ref1) < 1e-2
    assert rel_err(d2, ref2) < 1e-2


@pytest.mark.parametrize("N,H,C1,C2,Cout,tile", [
    (2, 128, 32, 0, 32, 6), (3, 128, 32, 32, 32, 6), (2, 64, 64, 0, 64, 6), (3, 64, 64, 64, 64, 6),
    (2, 64, 32, 0, 64, 6), (3, 16, 32, 0, 32, 6), (5, 16, 64, 0, 64, 6), (3, 32, 128, 0, 32, 6),
    (1, 128, 32, 0, 64, 0), (2, 64, 64, 64, 64, 0), (2, 32, 64, 0, 128, 8),
    (2, 128, 32, 0, 64, 12), (3, 128, 32, 32, 64, 12), (3, 64, 64, 64, 64, 12), (5, 16, 64, 0, 128, 12),
    (3, 32, 128, 0, 64, 12), (2, 16, 256, 256, 256, 12)])
def test_conv_row_window(cuda_dev, N, H, C1, C2, Cout, tile):
    """Row-window kernel (tile 6, auto for 16 <= W <= 128): image boundaries inside a window,
    row tails (N*H not a multiple of the window), concat sources, bias + ReLU + dropout."""
    torch.manual_seed(N * 100 + H + C1 + C2)
    a = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    b2 = torch.randn(N, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.08).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    out = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(b2) if C2 else None, wgt=ptr(pack_fwd(w)), bias=ptr(bias), Cout=Cout, relu=1,
                      dst1=ptr(out), tile=tile), stream())
    xin = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    ref = nhwc(F.relu(F.conv2d(xin, w.float().permute(3, 2, 0, 1), bias, padding=1)))
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,tile", [(2, 8, 256, 32, 0, 32, 6), (1, 4, 384, 32, 32, 32, 6),
                                                    (2, 8, 512, 64, 0, 64, 6), (1, 4, 256, 64, 64, 64, 6),
                                                    (2, 8, 512, 64, 0, 64, 12), (1, 4, 256, 64, 64, 128, 12)])
def test_conv_row_window_segmented_rows(cuda_dev, N, H, W, C1, C2, Cout, tile):
    """Rows wider than 128 run as 128-wide segments whose halo columns are the
    neighbouring segments' pixels (512x512 config levels)."""
    torch.manual_seed(N + H + W + C1 + C2)
    a = torch.randn(N, H, W, C1, device=cuda_dev).bfloat16()
    b2 = torch.randn(N, H, W, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.08).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    out = torch.empty(N, H, W, Cout, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(b2) if C2 else None, wgt=ptr(pack_fwd(w)), bias=ptr(bias), Cout=Cout, relu=1,
                      dst1=ptr(out), tile=tile), stream())
    xin = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    ref = nhwc(F.relu(F.conv2d(xin, w.float().permute(3, 2, 0, 1), bias, padding=1)))
    assert rel_err(out, ref) < 1e-2


def ncdhw(x):
    return x.permute(0, 4, 1, 2, 3)


def ndhwc(x):
    return x.permute(0, 2, 3, 4, 1)


@pytest.mark.parametrize("N,D,H,C1,C2,Cout", [(1, 4, 32, 32, 0, 32), (2, 3, 64, 32, 32, 32), (1, 2, 128, 64, 0, 64),
                                               (1, 4, 16, 64, 64, 128)])
def test_conv3d_row_window(cuda_dev, N, D, H, C1, C2, Cout):
    """3x3x3 conv on the row-window kernel: three depth taps, each a 9-tap window pass over
    the rows of slice d + dz - 1 (zero outside the volume); fwd + concat dgrad."""
    torch.manual_seed(N + D + H + C1)
    a = torch.randn(N, D, H, H, C1, device=cuda_dev).bfloat16()
    b2 = torch.randn(N, D, H, H, max(C2, 1), device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, 3, C1 + C2, Cout, device=cuda_dev) * 0.05).bfloat16()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    out = torch.empty(N, D, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
    wp = pad64(w.permute(4, 0, 1, 2, 3).reshape(Cout, -1))
    geo = dict(N=N, OD=D, OH=H, OW=H, ID=D, IH=H, IW=H, KD=3, KH=3, KW=3, pad=1)
    C().conv_fwd(dict(geo, C1=C1, C2=C2, src1=ptr(a), src2=ptr(b2) if C2 else None, wgt=ptr(wp), bias=ptr(bias),
                      Cout=Cout, relu=1, dst1=ptr(out), tile=6), stream())
    xin = ncdhw(a.float()) if not C2 else torch.cat([ncdhw(a.float()), ncdhw(b2.float())], 1)
    wt = w.float().permute(4, 3, 0, 1, 2)
    ref = ndhwc(F.relu(F.conv3d(xin, wt, bias, padding=1)))
    assert rel_err(out, ref) < 1e-2
    # dgrad: flipped taps, weights [ci][tap][co], split destinations, ReLU mask on src2
    dy = torch.randn(N, D, H, H, Cout, device=cuda_dev).bfloat16()
    wdg = pad64(w.flip(0, 1, 2).permute(3, 0, 1, 2, 4).reshape(C1 + C2, -1))
    d1 = torch.empty(N, D, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, D, H, H, max(C2, 1), device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(geo, C1=Cout, src1=ptr(dy), wgt=ptr(wdg), Cout=C1 + C2, D1=C1, dst1=ptr(d1),
                      dst2=ptr(d2) if C2 else None, mask2=ptr(b2) if C2 else None, tile=6), stream())
    xr = torch.zeros(N, C1 + C2, D, H, H, device=cuda_dev, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv3d(xr, wt, padding=1), xr, ncdhw(dy.float()))
    g = ndhwc(g)
    assert rel_err(d1, g[..., :C1]) < 1e-2
    if C2:
        assert rel_err(d2, g[..., C1:] * (b2.float() > 0)) < 1e-2


def test_conv_row_window_dgrad_dual_dest_mask_dropout(cuda_dev):
    """The row-window kernel as a concat dgrad (flipped weights, two destinations,
    ReLU mask + dropout rescale) at the 128-wide level."""
    torch.manual_seed(22)
    N, H, C1, C2, Co = 2, 128, 32, 32, 32
    skip = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
    m1 = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.1).bfloat16()
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    d1 = torch.empty(N, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    for tile in (6, 8, 12):
        C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy),
                          wgt=ptr(pack_dgrad(w)), Cout=C1 + C2, D1=C1, dst1=ptr(d1), dst2=ptr(d2),
                          mask1=ptr(m1), mask2=ptr(skip), mask_scale2=1.25, tile=tile), stream())
        xr = torch.zeros(N, C1 + C2, H, H, device=cuda_dev, requires_grad=True)
        y = F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1)
        (g,) = torch.autograd.grad(y, xr, nchw(dy.float()))
        g = nhwc(g)
        assert rel_err(d1, g[..., :C1] * (m1.float() > 0)) < 1e-2
        assert rel_err(d2, g[..., C1:] * (skip.float() > 0) * 1.25) < 1e-2


@pytest.mark.parametrize("N,H,Cin,Co,tile", [(2, 32, 4, 32, 0), (3, 128, 4, 32, 9), (5, 16, 4, 64, 9),
                                             (2, 64, 8, 32, 9), (2, 32, 4, 32, 8), (2, 32, 8, 64, 8),
                                             (9, 128, 4, 32, 9), (5, 32, 4, 32, 9), (3, 64, 4, 64, 9),
                                             (5, 32, 8, 64, 9), (2, 256, 4, 32, 9), (3, 512, 4, 32, 9),
                                             (2, 512, 8, 64, 9)])
def test_conv_first_layer_smallc(cuda_dev, N, H, Cin, Co, tile):
    """First layer (padded 4/8 channels): row-window kernel (tile 9, auto; 8 windows per
    workgroup with the next halo prefetched -- full and partial groups, 1-2 channel
    tiles; rows 16..512 wide, a window of one 512-wide row) and the implicit-GEMM small-C
    mode (tile 8)."""
    torch.manual_seed(3)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Co, device=cuda_dev) * 0.2).bfloat16()
    b = torch.randn(Co, device=cuda_dev)
    wp = pack_fwd(w)
    out = torch.empty(N, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp),
                      bias=ptr(b), Cout=Co, relu=1, dst1=ptr(out), tile=tile), stream())
    ref = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("N,D,H,Cin,Co,tile", [(1, 4, 32, 4, 32, 9), (2, 3, 64, 4, 64, 9), (1, 5, 128, 8, 32, 9),
                                               (1, 4, 32, 4, 32, 0), (1, 3, 32, 4, 32, 8)])
def test_conv3d_first_layer_window(cuda_dev, N, D, H, Cin, Co, tile):
    """3D first layer (padded 4/8 channels) on the first-layer window (tile 9 / auto): per
    depth tap the halo of slice d + kd - 1 (zeros past the volume) and that tap's weights,
    the next (window, depth tap)'s halo prefetched; tile 8 = the implicit-GEMM small-C mode."""
    torch.manual_seed(D + H + Cin)
    x = torch.randn(N, D, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, 3, Cin, Co, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Co, device=cuda_dev)
    wp = pad64(w.permute(4, 0, 1, 2, 3).reshape(Co, -1))
    out = torch.empty(N, D, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OD=D, OH=H, OW=H, ID=D, IH=H, IW=H, KD=3, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x),
                      wgt=ptr(wp), bias=ptr(b), Cout=Co, relu=1, dst1=ptr(out), tile=tile), stream())
    ref = ndhwc(F.relu(F.conv3d(ncdhw(x.float()), w.float().permute(4, 3, 0, 1, 2), b, padding=1)))
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("N,H,Ci,Co,tile", [(2, 8, 64, 32, 0), (2, 8, 64, 32, 8), (3, 64, 64, 32, 0),
                                            (2, 32, 128, 64, 0), (5, 16, 256, 128, 0), (3, 8, 512, 256, 0),
                                            (2, 128, 128, 64, 0), (1, 256, 64, 32, 0), (1, 512, 64, 32, 0)])
def test_tconv_fwd_shuffle_and_dgrad(cuda_dev, N, H, Ci, Co, tile):
    """2x2 stride-2 transposed conv: window kernels (auto) and the implicit-GEMM path (tile 8)."""
    torch.manual_seed(4)
    x = F.relu(torch.randn(N, H, H, Ci, device=cuda_dev)).bfloat16()
    k = (torch.randn(2, 2, Co, Ci, device=cuda_dev) * 0.1).bfloat16()   # Keras (kh,kw,Cout,Cin)
    b = torch.randn(Co, device=cuda_dev)
    out = torch.empty(N, 2 * H, 2 * H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, C1=Ci, src1=ptr(x), wgt=ptr(pad64(k.reshape(4 * Co, Ci))),
                      bias=ptr(b), Cout=4 * Co, shuffle=2, dst1=ptr(out), tile=tile), stream())
    wt = k.float().permute(3, 2, 0, 1)      # (Cin, Cout, kh, kw)
    ref = nhwc(F.conv_transpose2d(nchw(x.float()), wt, b, stride=2))
    assert rel_err(out, ref) < 1e-2
    # dgrad: 2x2 stride-2 conv of dOut with weights [ci][tap][co], masked by x > 0
    dout = torch.randn(N, 2 * H, 2 * H, Co, device=cuda_dev).bfloat16()
    wdg = pad64(k.permute(3, 0, 1, 2).reshape(Ci, 4 * Co))
    dx = torch.empty(N, H, H, Ci, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=2 * H, IW=2 * H, KH=2, KW=2, stride=2, pad=0, C1=Co,
                      src1=ptr(dout), wgt=ptr(wdg), Cout=Ci, dst1=ptr(dx), mask1=ptr(x), tile=tile), stream())
    xr = nchw(x.float()).requires_grad_(True)
    (g,) = torch.autograd.grad(F.conv_transpose2d(xr, wt, stride=2), xr, nchw(dout.float()))
    ref = nhwc(g) * (x.float() > 0)
    assert rel_err(dx, ref) < 1e-2


def _wgrad(d, splits, taps, Mtot, Mout, Nc, out_numel, bias_w=None, rows=None):
    dev = torch.device("cuda")
    slab = torch.zeros(splits * taps * Mtot * Nc, device=dev)
    bslab = torch.zeros(splits * 8 * max(Mtot, Nc), device=dev)
    d = dict(d, splits=splits, slab=ptr(slab), bias_slab=ptr(bslab))
    C().wgrad(d, stream())
    out = torch.zeros(out_numel, device=dev)
    stage = torch.zeros(C().wgrad_reduce_stage_floats(max(splits, 64), taps, Mtot, Nc) + 4096, device=dev)
    ints = [splits, taps, Mtot, Mout, Nc] + (list(rows) if rows else [])
    C().generic("wgrad_reduce", [ptr(slab), ptr(out), ptr(stage)], ints, [1.0], stream())
    bout = None
    if bias_w is not None:
        nrows, w = bias_w
        bout = torch.zeros(w, device=dev)
        C().generic("wgrad_reduce", [ptr(bslab), ptr(bout), ptr(stage)], [nrows, 1, 1, 1, w], [1.0], stream())
    return out, bout


@pytest.mark.parametrize("N,H,Cin,Cout,splits", [(4, 16, 32, 32, 3), (8, 32, 32, 32, 40), (2, 16, 64, 128, 2), (2, 8, 128, 128, 4),
                                                  (2, 8, 256, 512, 2)])
def test_conv_wgrad_and_bias(cuda_dev, N, H, Cin, Cout, splits):
    torch.manual_seed(5)
    x = F.relu(torch.randn(N, H, H, Cin, device=cuda_dev)).bfloat16()
    dy = torch.randn(N, H, H, Cout, device=cuda_dev).bfloat16()
    BM, BN, NTAP, smallc = C().wgrad_pick(Cin, 0, Cout, 9)
    d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=Cin, a1=ptr(x), b=ptr(dy), Nc=Cout,
             bias_mode=1)
    gw, gb = _wgrad(d, splits, 9, Cin, Cin, Cout, 9 * Cin * Cout, bias_w=(splits, Cout))
    w = torch.zeros(Cout, Cin, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    y = F.conv2d(nchw(x.float()), w, bb, padding=1)
    gwr, gbr = torch.autograd.grad(y, [w, bb], nchw(dy.float()))
    ref = gwr.permute(2, 3, 1, 0).reshape(-1)        # HWIO
    assert rel_err(gw, ref) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,H,C1,C2,Cout,splits,win", [
    (3, 128, 32, 0, 32, 5, 0), (2, 128, 32, 32, 32, 7, 0), (4, 64, 64, 0, 64, 3, 0), (3, 64, 64, 64, 64, 9, 0),
    (2, 64, 32, 0, 64, 2, 0), (5, 32, 64, 0, 128, 4, 0), (2, 32, 128, 128, 128, 3, 0), (3, 32, 32, 0, 32, 40, 0),
    (2, 64, 64, 0, 64, 3, -1), (4, 16, 64, 0, 64, 3, 0), (3, 16, 128, 128, 128, 5, 0), (4, 8, 256, 0, 256, 2, 0),
    (3, 8, 32, 0, 32, 7, 0)])
def test_wgrad_row_window(cuda_dev, N, H, C1, C2, Cout, splits, win):
    """Row-window wgrad (auto for 2D 3x3 on 32..128-wide rows): concat sources, 32/64-wide
    output-channel blocks, more splits than windows, fused bias sums; win=-1 = tiled kernel."""
    torch.manual_seed(N + H + C1 + C2 + Cout)
    a = F.relu(torch.randn(N, H, H, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(N, H, H, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(N, H, H, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=C1, M2=C2, a1=ptr(a),
             a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1, win=win)
    gw, gb = _wgrad(d, splits, 9, Mt, Mt, Cout, 9 * Mt * Cout, bias_w=(splits, Cout))
    inp = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    w = torch.zeros(Cout, Mt, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(inp, w, bb, padding=1), [w, bb], nchw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,splits", [(2, 4, 256, 32, 0, 32, 3), (1, 6, 384, 32, 32, 32, 4),
                                                      (2, 4, 512, 64, 0, 64, 5), (1, 4, 256, 64, 64, 64, 2)])
def test_wgrad_row_window_segmented_rows(cuda_dev, N, H, W, C1, C2, Cout, splits):
    """Window wgrad on rows wider than 128 (128-wide segments, neighbour halo columns)."""
    torch.manual_seed(N + H + W + C1 + C2)
    a = F.relu(torch.randn(N, H, W, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(N, H, W, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(N, H, W, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    assert C().wgrad_pick(C1, C2, Cout, 9, QW=W, QH=H, win=0)[2] == 9      # window tile picked
    d = dict(N=N, QH=H, QW=W, AH=H, AW=W, KH=3, KW=3, pad=1, M1=C1, M2=C2, a1=ptr(a),
             a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1)
    gw, gb = _wgrad(d, splits, 9, Mt, Mt, Cout, 9 * Mt * Cout, bias_w=(splits, Cout))
    inp = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    w = torch.zeros(Cout, Mt, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(inp, w, bb, padding=1), [w, bb], nchw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,D,H,C1,C2,Cout,splits", [(1, 4, 32, 32, 0, 32, 3), (2, 3, 64, 32, 32, 32, 5),
                                                      (1, 2, 128, 64, 0, 64, 2), (1, 4, 32, 64, 64, 128, 7)])
def test_wgrad3d_row_window(cuda_dev, N, D, H, C1, C2, Cout, splits):
    """3x3x3 wgrad on the window kernel: one tap group per depth tap (27-tap slab)."""
    torch.manual_seed(N + D + H + C1 + C2)
    a = F.relu(torch.randn(N, D, H, H, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(N, D, H, H, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(N, D, H, H, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    assert C().wgrad_pick(C1, C2, Cout, 27, QW=H, QH=H, QD=D, win=0)[2] == 9
    d = dict(N=N, QD=D, QH=H, QW=H, AD=D, AH=H, AW=H, KD=3, KH=3, KW=3, pad=1, M1=C1, M2=C2, a1=ptr(a),
             a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1)
    gw, gb = _wgrad(d, splits, 27, Mt, Mt, Cout, 27 * Mt * Cout, bias_w=(splits, Cout))
    inp = ncdhw(a.float()) if not C2 else torch.cat([ncdhw(a.float()), ncdhw(b2.float())], 1)
    w = torch.zeros(Cout, Mt, 3, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv3d(inp, w, bb, padding=1), [w, bb], ncdhw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 4, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,H,Creal,Cpad,Co,splits,win", [(2, 32, 1, 4, 32, 3, -1), (2, 32, 1, 4, 32, 3, 0),
                                                           (3, 128, 4, 4, 32, 7, 0), (2, 16, 3, 4, 64, 40, 0),
                                                           (2, 64, 8, 8, 32, 5, 0), (2, 32, 5, 8, 32, 3, -1),
                                                           (2, 256, 1, 4, 32, 6, 0), (2, 512, 4, 4, 32, 9, 0),
                                                           (1, 512, 8, 8, 64, 4, 0)])
def test_wgrad_first_layer_smallc(cuda_dev, N, H, Creal, Cpad, Co, splits, win):
    """First-layer weight gradient: row-window kernel (win=0) and the tiled small-C mode
    (win=-1); padded channels dropped by the slab reduction's row remap."""
    torch.manual_seed(7)
    x = torch.zeros(N, H, H, Cpad, device=cuda_dev)
    x[..., :Creal] = torch.randn(N, H, H, Creal, device=cuda_dev)
    x = x.bfloat16()
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    BM, BN, NTAP, smallc = C().wgrad_pick(Cpad, 0, Co, 9, QW=H, win=win)
    assert smallc
    Mtot = (9 * Cpad + BM - 1) // BM * BM
    d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=Cpad, a1=ptr(x), b=ptr(dy), Nc=Co,
             bias_mode=1, win=win)
    gw, gb = _wgrad(d, splits, 1, Mtot, 9 * Creal, Co, 9 * Creal * Co, bias_w=(splits, Co), rows=(Cpad, Creal))
    w = torch.zeros(Co, Creal, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Co, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(nchw(x.float()[..., :Creal]), w, bb, padding=1), [w, bb],
                                   nchw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,D,H,Creal,Co,splits,win", [(1, 4, 32, 4, 32, 3, 0), (2, 3, 64, 1, 32, 5, 0),
                                                         (1, 5, 128, 4, 64, 7, 0), (1, 4, 32, 4, 32, 3, -1)])
def test_wgrad_first_layer_3d(cuda_dev, N, D, H, Creal, Co, splits, win):
    """3D first-layer weight gradient (4 padded channels): the window kernel staging the three
    depth slices' halos (win = 0) and the tiled small-C mode (win = -1), rows remapped like
    the engine's (taps x padded channels -> taps x real channels)."""
    torch.manual_seed(9)
    Cpad = 4
    x = torch.zeros(N, D, H, H, Cpad, device=cuda_dev)
    x[..., :Creal] = torch.randn(N, D, H, H, Creal, device=cuda_dev)
    x = x.bfloat16()
    dy = torch.randn(N, D, H, H, Co, device=cuda_dev).bfloat16()
    BM, BN, NTAP, smallc = C().wgrad_pick(Cpad, 0, Co, 27, QW=H, win=win, QH=H, QD=D)
    assert smallc
    Mtot = (27 * Cpad + BM - 1) // BM * BM
    d = dict(N=N, QD=D, QH=H, QW=H, AD=D, AH=H, AW=H, KD=3, KH=3, KW=3, pad=1, M1=Cpad, a1=ptr(x), b=ptr(dy),
             Nc=Co, bias_mode=1, win=win)
    gw, gb = _wgrad(d, splits, 1, Mtot, 27 * Creal, Co, 27 * Creal * Co, bias_w=(splits, Co), rows=(Cpad, Creal))
    w = torch.zeros(Co, Creal, 3, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Co, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv3d(ncdhw(x.float()[..., :Creal]), w, bb, padding=1), [w, bb],
                                   ncdhw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 4, 1, 0).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,H,Ci,Co,splits,win", [(2, 8, 64, 32, 2, 0), (3, 64, 64, 32, 5, 0), (2, 32, 128, 64, 3, 0),
                                                   (2, 32, 128, 64, 3, -1), (3, 64, 64, 32, 40, 0)])
def test_tconv_wgrad_bias_mode2(cuda_dev, N, H, Ci, Co, splits, win):
    """Transposed-conv weight + bias gradients: window kernel (coarse rows 32/64, auto) and
    the tiled kernel; the slab / bias-slab layout comes from wgrad_pick like the engine."""
    torch.manual_seed(8)
    x = F.relu(torch.randn(N, H, H, Ci, device=cuda_dev)).bfloat16()
    dout = torch.randn(N, 2 * H, 2 * H, Co, device=cuda_dev).bfloat16()
    d = dict(N=N, QH=H, QW=H, AH=2 * H, AW=2 * H, KH=2, KW=2, stride=2, pad=0, M1=Co, a1=ptr(dout),
             b=ptr(x), Nc=Ci, bias_mode=2, win=win)
    BM, BN, NTAP, _ = C().wgrad_pick(Co, 0, Ci, 4, QW=H, win=win)
    tg = 4 // NTAP
    gw, gb = _wgrad(d, splits, 4, Co, Co, Ci, 4 * Co * Ci, bias_w=(splits * tg, Co))
    k = torch.zeros(Ci, Co, 2, 2, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Co, device=cuda_dev, requires_grad=True)
    gk, gbr = torch.autograd.grad(F.conv_transpose2d(nchw(x.float()), k, bb, stride=2), [k, bb],
                                  nchw(dout.float()))
    ref = gk.permute(2, 3, 1, 0).reshape(-1)     # (kh, kw, Cout, Cin)
    assert rel_err(gw, ref) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


def test_maxpool_fwd_bwd_with_skip(cuda_dev):
    torch.manual_seed(9)
    N, H, Cc = 2, 16, 32
    x = F.relu(torch.randn(N, H, H, Cc, device=cuda_dev)).bfloat16()
    y = torch.empty(N, H // 2, H // 2, Cc, device=cuda_dev, dtype=torch.bfloat16)
    C().generic("pool_fwd", [ptr(x), ptr(y)], [N, 1, H, H, Cc, 0], [], stream())
    ref = nhwc(F.max_pool2d(nchw(x.float()), 2))
    assert (y.float() - ref).abs().max().item() == 0
    dy = torch.randn_like(y.float()).bfloat16()
    skip = torch.randn_like(x.float()).bfloat16()
    dx = torch.empty_like(x)
    C().generic("pool_bwd", [ptr(x), ptr(dy), ptr(skip), ptr(dx)], [N, 1, H, H, Cc, 0], [], stream())
    xr = nchw(x.float()).requires_grad_(True)
    (g,) = torch.autograd.grad(F.max_pool2d(xr, 2), xr, nchw(dy.float()))
    # the pool backward includes the derivative of the ReLU that produced x: a window
    # whose inputs are all clipped (max 0) routes nothing
    assert rel_err(dx, nhwc(g) * (x.float() > 0) + skip.float()) < 1e-2


def test_head_fwd_bwd(cuda_dev):
    torch.manual_seed(10)
    P, Cc = 4096, 32
    x = F.relu(torch.randn(P, Cc, device=cuda_dev)).bfloat16()
    w = torch.randn(Cc, device=cuda_dev) * 0.3
    b = torch.randn(1, device=cuda_dev)
    t = (torch.rand(P, device=cuda_dev) > 0.7).bfloat16()
    prob = torch.empty(P, device=cuda_dev)
    nb = C().head_blocks(P)
    part = torch.empty(nb * (Cc + 1) + 4 * nb, device=cuda_dev)
    sums = torch.empty(4, device=cuda_dev)
    C().generic("head_fwd", [ptr(x), ptr(w), ptr(b), ptr(t), ptr(prob), ptr(part), ptr(sums)], [P, Cc], [],
                stream())
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    z = xr @ wr + br
    p = torch.sigmoid(z)
    tf = t.float()
    I, St, Sp = (tf * p).sum(), tf.sum(), p.sum()
    bce = F.binary_cross_entropy_with_logits(z, tf, reduction="sum")
    assert rel_err(prob, p) < 1e-4
    assert rel_err(sums, torch.stack([I, St, Sp, bce])) < 1e-4
    loss = -torch.log(2 * I + 1) + torch.log(St + Sp + 1) + 0.5 * bce / P
    gx, gw, gb = torch.autograd.grad(loss, [xr, wr, br])
    dx = torch.empty_like(x)
    ow = torch.empty(Cc, device=cuda_dev)
    ob = torch.empty(1, device=cuda_dev)
    C().generic("head_bwd", [ptr(x), ptr(w), ptr(prob), ptr(t), ptr(sums), ptr(dx), ptr(part), ptr(ow),
                             ptr(ob)], [P, Cc], [1.0 / P, 0.5, 1.0], stream())
    assert rel_err(dx, gx * (x.float() > 0)) < 1e-2
    assert rel_err(ow, gw) < 1e-3
    assert rel_err(ob, gb) < 1e-3


def test_dropout_matches_reference_hash(cuda_dev):
    from unet_distributed_amd.models.reference import dropout_keep_mask
    torch.manual_seed(11)
    N, H, Cin, Co = 2, 8, 32, 64
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Co, device=cuda_dev) * 0.1).bfloat16()
    out = torch.empty(N, H, H, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x),
                      wgt=ptr(pack_fwd(w)), Cout=Co, relu=1, dst1=ptr(out), drop_rate=0.2, seed=1234, salt=7),
                 stream())
    keep = dropout_keep_mask(1234, 7, out.shape, 0.2, cuda_dev)
    ref = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), padding=1))) * keep / 0.8
    assert rel_err(out, ref) < 1e-2
    frac = keep.float().mean().item()
    assert 0.75 < frac < 0.85


@pytest.mark.parametrize("norm,N,H,Cc,G", [("batch", 4, 16, 32, 0), ("batch", 3, 8, 64, 0), ("group", 4, 16, 64, 8),
                                           ("group", 2, 8, 32, 4), ("batch", 80, 4, 32, 0), ("group", 70, 4, 48, 4),
                                           ("batch", 2, 32, 48, 0)])
def test_norm_fwd_bwd_kernels(cuda_dev, norm, N, H, Cc, G):
    """BN / GN forward (batch statistics, ReLU) and backward (dz, dgamma, dbeta) against
    autograd of the fp32 ATen ops on the same bf16 inputs."""
    torch.manual_seed(31)
    dev = cuda_dev
    P = H * H
    z = (torch.randn(N, H, H, Cc, device=dev) * 2 + 0.5).bfloat16()
    gam = torch.rand(Cc, device=dev) + 0.5
    bet = torch.randn(Cc, device=dev) * 0.1
    g = torch.randn(N, H, H, Cc, device=dev).bfloat16()
    nbp = C().norm_blocks_per_sample(N, P)
    part = torch.zeros(N * nbp * 2 * Cc, device=dev)
    S = torch.zeros(N * 2 * Cc, device=dev)
    rows = 1 if norm == "batch" else N
    mean, rstd, ca, cb, cc = [torch.zeros(rows * Cc, device=dev) for _ in range(5)]
    rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
    dg, db = torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev)
    work = torch.zeros(C().sample_slices(N) * 2 * Cc, device=dev)        # finalize workspace
    wp = ptr(work)
    y = torch.empty_like(z)
    dz = torch.empty_like(z)
    st = stream()
    C().generic("norm_moments", [ptr(z), ptr(z), ptr(part), ptr(S)], [N, P, Cc], [], st)
    if norm == "batch":
        C().generic("bn_finalize", [ptr(S), ptr(gam), ptr(rm), ptr(rv), ptr(mean), ptr(rstd), 0, 0, 0, 0, 0, wp],
                    [N, Cc, 0], [float(N * P), 1e-3, 0.01], st)
        cs = 0
    else:
        C().generic("gn_finalize", [ptr(S), ptr(gam), ptr(mean), ptr(rstd), 0, 0, 0, 0, 0, wp], [N, Cc, G, P, 0],
                    [1e-3], st)
        cs = Cc
    C().generic("norm_apply", [ptr(z), ptr(mean), ptr(rstd), ptr(gam), ptr(bet), ptr(y)], [N, P, Cc, cs, 1, 0, 0],
                [0.0], st)
    C().generic("norm_moments", [ptr(g), ptr(z), ptr(part), ptr(S)], [N, P, Cc], [], st)
    if norm == "batch":
        C().generic("bn_finalize", [ptr(S), ptr(gam), 0, 0, ptr(mean), ptr(rstd), ptr(ca), ptr(cb), ptr(cc), ptr(dg),
                                    ptr(db), wp], [N, Cc, 1], [float(N * P), 1e-3, 0.01], st)
    else:
        C().generic("gn_finalize", [ptr(S), ptr(gam), ptr(mean), ptr(rstd), ptr(ca), ptr(cb), ptr(cc), ptr(dg),
                                    ptr(db), wp], [N, Cc, G, P, 1], [1e-3], st)
    C().generic("norm_bwd_apply", [ptr(g), ptr(z), ptr(ca), ptr(cb), ptr(cc), ptr(dz)], [N, P, Cc, cs], [], st)
    torch.cuda.synchronize()
    zr = nchw(z.float()).requires_grad_(True)
    gr = gam.clone().requires_grad_(True)
    br = bet.clone().requires_grad_(True)
    if norm == "batch":
        rmr, rvr = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
        o = F.batch_norm(zr, rmr, rvr, gr, br, training=True, momentum=0.01, eps=1e-3)
    else:
        o = F.group_norm(zr, G, gr, br, eps=1e-3)
    # the kernel's bwd input g is dL/d(norm output) already ReLU-masked by the consumer
    yref = F.relu(o)
    dzr, dgr, dbr = torch.autograd.grad(o, [zr, gr, br], nchw(g.float()))
    assert rel_err(y, nhwc(yref)) < 1e-2
    assert rel_err(dz, nhwc(dzr)) < 2e-2
    assert rel_err(dg, dgr) < 1e-3 and rel_err(db, dbr) < 1e-3
    if norm == "batch":
        assert torch.allclose(rm, rmr, atol=1e-5) and torch.allclose(rv, rvr, atol=1e-4)


@pytest.mark.parametrize("dims3", [0, 1])
def test_maxpool_argmax_codes_match_recomputed_argmax(cuda_dev, dims3):
    """pool_fwd's first-argmax codes drive the same backward as recomputing the argmax
    from the input (ReLU zeros make ties: the FIRST maximum wins in both)."""
    torch.manual_seed(19)
    N, D, H, Cc = 2, (4 if dims3 else 1), 16, 32
    shape = (N, D, H, H, Cc) if dims3 else (N, H, H, Cc)
    x = F.relu(torch.randn(*shape, device=cuda_dev)).bfloat16()
    oshape = (N, D // 2, H // 2, H // 2, Cc) if dims3 else (N, H // 2, H // 2, Cc)
    y = torch.empty(*oshape, device=cuda_dev, dtype=torch.bfloat16)
    code = torch.full((y.numel() // 8,), -1, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(x), ptr(y), ptr(code)], [N, D, H, H, Cc, dims3], [], stream())
    if dims3:
        ref = F.max_pool3d(x.float().permute(0, 4, 1, 2, 3), 2).permute(0, 2, 3, 4, 1)
    else:
        ref = nhwc(F.max_pool2d(nchw(x.float()), 2))
    assert (y.float() - ref).abs().max().item() == 0
    dy = torch.randn_like(y.float()).bfloat16()
    skip = torch.randn_like(x.float()).bfloat16()
    dx_x, dx_c = torch.empty_like(x), torch.empty_like(x)
    C().generic("pool_bwd", [ptr(x), ptr(dy), ptr(skip), ptr(dx_x)], [N, D, H, H, Cc, dims3], [], stream())
    C().generic("pool_bwd", [0, ptr(dy), ptr(skip), ptr(dx_c), ptr(code)], [N, D, H, H, Cc, dims3], [], stream())
    torch.cuda.synchronize()
    assert torch.equal(dx_x, dx_c)


@pytest.mark.parametrize("dims3", [0, 1])
def test_upsample2_fwd_materialised(cuda_dev, dims3):
    """Nearest x2 upsample (the upsampling decoder's materialised source) is exact."""
    torch.manual_seed(23)
    N, D, H, Cc = 2, (3 if dims3 else 1), 8, 64
    shape = (N, D, H, H, Cc) if dims3 else (N, H, H, Cc)
    x = torch.randn(*shape, device=cuda_dev).bfloat16()
    ref = x.repeat_interleave(2, -2).repeat_interleave(2, -3)
    if dims3:
        ref = ref.repeat_interleave(2, 1)
    y = torch.empty_like(ref)
    C().generic("ups_fwd", [ptr(x), ptr(y)], [N, D, H, H, Cc, dims3], [], stream())
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("N,H,Cin,Cout,tile", [(2, 128, 32, 32, 0), (2, 64, 32, 64, 0), (4, 32, 64, 128, 0),
                                               (4, 16, 128, 256, 0), (1, 256, 32, 32, 0), (2, 128, 32, 64, 12),
                                               (2, 64, 32, 64, 12), (4, 32, 64, 128, 12), (4, 16, 128, 256, 12)])
def test_conv_fwd_fused_maxpool_matches_pool_kernel(cuda_dev, N, H, Cin, Cout, tile):
    """convNb forward with the fused 2x2 max-pool epilogue: the conv output, the pooled
    tensor and the argmax codes equal the plain conv + the separate pool kernel."""
    torch.manual_seed(31)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    y0, y1 = [torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16) for _ in range(2)]
    p0, p1 = [torch.empty(N, H // 2, H // 2, Cout, device=cuda_dev, dtype=torch.bfloat16) for _ in range(2)]
    c0, c1 = [torch.full((N * (H // 2) ** 2 * Cout // 8,), -1, device=cuda_dev, dtype=torch.int32) for _ in range(2)]
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp), bias=ptr(b),
             Cout=Cout, relu=1, tile=tile)
    C().conv_fwd(dict(d, dst1=ptr(y0)), stream())
    C().generic("pool_fwd", [ptr(y0), ptr(p0), ptr(c0)], [N, 1, H, H, Cout, 0], [], stream())
    C().conv_fwd(dict(d, dst1=ptr(y1), pool_dst=ptr(p1), pool_code=ptr(c1)), stream())
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(p0, p1)
    assert torch.equal(c0, c1)


def _pack_bits(y):
    """[..., C] activation -> [..., C / 8] uint8, bit e of byte b = channel 8b + e > 0."""
    pos = (y.float() > 0).to(torch.int32).reshape(*y.shape[:-1], y.shape[-1] // 8, 8)
    return (pos << torch.arange(8, device=y.device, dtype=torch.int32)).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("N,H,Cin,Cout,tile,drop", [(2, 128, 32, 32, 0, 0.0), (2, 64, 32, 64, 0, 0.0),
                                                    (4, 16, 128, 256, 0, 0.0), (2, 32, 64, 64, 8, 0.0),
                                                    (2, 128, 4, 32, 9, 0.0), (2, 16, 64, 128, 0, 0.3)])
def test_conv_fwd_relu_bits(cuda_dev, N, H, Cin, Cout, tile, drop):
    """A ReLU forward (row-window, implicit-GEMM, first-layer, dropout / generic
    epilogue) also writes the 1-bit-per-element mask of its stored output, and the
    output itself is unchanged."""
    torch.manual_seed(41)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cout, device=cuda_dev) * 0.1
    wp = pack_fwd(w)
    y0, y1 = [torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16) for _ in range(2)]
    bits = torch.full((N, H, H, Cout // 8), 0xA5, device=cuda_dev, dtype=torch.uint8)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp), bias=ptr(b),
             Cout=Cout, relu=1, drop_rate=drop, seed=5, salt=3, tile=tile)
    C().conv_fwd(dict(d, dst1=ptr(y0)), stream())
    C().conv_fwd(dict(d, dst1=ptr(y1), relu_bits=ptr(bits)), stream())
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(bits, _pack_bits(y1))


@pytest.mark.parametrize("tile", [6, 8, 12])
def test_conv_dgrad_bit_masks_match_activation_masks(cuda_dev, tile):
    """Data gradient with two destinations whose ReLU masks come from bit tensors
    (mask_bits) equals the same launch masked by the 16-bit activations."""
    torch.manual_seed(42)
    N, H, C1, C2, Co = 2, 64, 32, 32, 32
    skip = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
    m1 = torch.randn(N, H, H, C1, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.1).bfloat16()
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    outs = []
    for bits in (False, True):
        d1 = torch.empty(N, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
        d2 = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
        mk1 = _pack_bits(m1) if bits else m1
        mk2 = _pack_bits(skip) if bits else skip
        C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy),
                          wgt=ptr(pack_dgrad(w)), Cout=C1 + C2, D1=C1, dst1=ptr(d1), dst2=ptr(d2),
                          mask1=ptr(mk1), mask2=ptr(mk2), mask_bits=3 if bits else 0, mask_scale2=1.25,
                          tile=tile), stream())
        torch.cuda.synchronize()
        outs.append((d1, d2))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("H,Ci,Co,tile", [(32, 64, 32, 0), (8, 512, 256, 0), (32, 64, 32, 8)])
def test_tconv_dgrad_bit_mask(cuda_dev, H, Ci, Co, tile):
    """Transposed-conv data gradient (window and implicit-GEMM kernels) with its ReLU
    mask read from a bit tensor."""
    torch.manual_seed(43)
    N = 2
    x = torch.randn(N, H, H, Ci, device=cuda_dev).bfloat16()
    k = (torch.randn(2, 2, Co, Ci, device=cuda_dev) * 0.1).bfloat16()
    dout = torch.randn(N, 2 * H, 2 * H, Co, device=cuda_dev).bfloat16()
    wdg = pad64(k.permute(3, 0, 1, 2).reshape(Ci, 4 * Co))
    res = []
    for bits in (False, True):
        dx = torch.empty(N, H, H, Ci, device=cuda_dev, dtype=torch.bfloat16)
        mk = _pack_bits(x) if bits else x
        C().conv_fwd(dict(N=N, OH=H, OW=H, IH=2 * H, IW=2 * H, KH=2, KW=2, stride=2, pad=0, C1=Co,
                          src1=ptr(dout), wgt=ptr(wdg), Cout=Ci, dst1=ptr(dx), mask1=ptr(mk),
                          mask_bits=int(bits), tile=tile), stream())
        torch.cuda.synchronize()
        res.append(dx)
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("N,H,C1,C2,Co", [(2, 128, 32, 32, 32), (2, 64, 64, 64, 64), (4, 32, 128, 128, 128),
                                          (4, 16, 256, 256, 256)])
def test_dgrad_skip_half_with_fused_pool_backward(cuda_dev, N, H, C1, C2, Co):
    """Decoder conv data gradient split in two: the upsampled half alone, and the skip
    half later with the max-pool backward in its epilogue (route_gy) -- equal, bit for
    bit, to the dual-destination dgrad + the separate argmax-code pool backward."""
    torch.manual_seed(44)
    y = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()        # convNb output (skip source)
    pooled = torch.empty(N, H // 2, H // 2, C2, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * C2 // 8, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, C2, 0], [], stream())
    dpool = torch.randn(N, H // 2, H // 2, C2, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=cuda_dev) * 0.1).bfloat16()
    wdg = pack_dgrad(w)                                  # [C1 + C2][9 Co pad 64]
    dy = torch.randn(N, H, H, Co, device=cuda_dev).bfloat16()
    bits = _pack_bits(y)
    geo = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy))
    # reference path: both halves in one dgrad, then the pool backward
    d_up0 = torch.empty(N, H, H, C1, device=cuda_dev, dtype=torch.bfloat16)
    dskip = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    dy0 = torch.empty(N, H, H, C2, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(geo, wgt=ptr(wdg), Cout=C1 + C2, D1=C1, dst1=ptr(d_up0), dst2=ptr(dskip), mask2=ptr(bits),
                      mask_bits=2), stream())
    C().generic("pool_bwd", [ptr(y), ptr(dpool), ptr(dskip), ptr(dy0), ptr(codes)], [N, 1, H, H, C2, 0], [],
                stream())
    # split path
    d_up1 = torch.empty_like(d_up0)
    dy1 = torch.empty_like(dy0)
    C().conv_fwd(dict(geo, wgt=ptr(wdg), Cout=C1, dst1=ptr(d_up1)), stream())
    C().conv_fwd(dict(geo, wgt=ptr(wdg) + 2 * C1 * wdg.shape[1], Cout=C2, dst1=ptr(dy1), mask1=ptr(bits),
                      mask_bits=1, route_gy=ptr(dpool), pool_code=ptr(codes)), stream())
    torch.cuda.synchronize()
    assert torch.equal(d_up0, d_up1)
    assert torch.equal(dy0, dy1)
    assert dy1.float().abs().sum() > 0


@pytest.mark.parametrize("kind", ["first", "win", "tconv"])
def test_wgrad_split_ranges_compose(cuda_dev, kind):
    """A weight gradient issued in parts (split_lo / split_n, e.g. the first layer's
    wgrad halves overlapping the last dgrad) writes exactly the slab rows of one
    launch over all splits."""
    torch.manual_seed(45)
    N, H = 4, 32
    if kind == "first":
        a = torch.randn(N, H, H, 4, device=cuda_dev).bfloat16()
        bt = torch.randn(N, H, H, 32, device=cuda_dev).bfloat16()
        d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=4, a1=ptr(a), b=ptr(bt), Nc=32, bias_mode=1)
        BM = C().wgrad_pick(4, 0, 32, 9, QW=H, win=0)[0]
        rows = (9 * 4 + BM - 1) // BM * BM * 32
    elif kind == "win":
        a = torch.randn(N, H, H, 64, device=cuda_dev).bfloat16()
        bt = torch.randn(N, H, H, 64, device=cuda_dev).bfloat16()
        d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=64, a1=ptr(a), b=ptr(bt), Nc=64, bias_mode=1)
        rows = 9 * 64 * 64
    else:
        a = torch.randn(N, 2 * H, 2 * H, 32, device=cuda_dev).bfloat16()     # dOut (fine)
        bt = torch.randn(N, H, H, 64, device=cuda_dev).bfloat16()            # layer input (coarse)
        d = dict(N=N, QH=H, QW=H, AH=2 * H, AW=2 * H, KH=2, KW=2, stride=2, pad=0, M1=32, a1=ptr(a), b=ptr(bt),
                 Nc=64, bias_mode=2)
        rows = 4 * 32 * 64
    splits = 6
    outs = []
    for parts in ([(0, 0)], [(0, 3), (3, 3)], [(0, 2), (2, 1), (3, 0)]):
        slab = torch.full((splits * rows,), float("nan"), device=cuda_dev)
        bslab = torch.full((splits * 8 * 64,), float("nan"), device=cuda_dev)
        for lo, n in parts:
            C().wgrad(dict(d, splits=splits, split_lo=lo, split_n=n, slab=ptr(slab), bias_slab=ptr(bslab)), stream())
        torch.cuda.synchronize()
        outs.append(slab)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("N,H,Cin,Cout,tile", [(2, 128, 32, 32, 0), (4, 32, 64, 128, 0), (4, 16, 128, 256, 0),
                                               (2, 256, 32, 32, 0)])
def test_window_conv_reverse_order_same_result(cuda_dev, N, H, Cin, Cout, tile):
    """rev = 1 (windows walked last to first: the consumer starts on its producer's
    most recent output) writes exactly the rev = 0 tensors, fused pool and ReLU bits
    included."""
    torch.manual_seed(46)
    x = torch.randn(N, H, H, Cin, device=cuda_dev).bfloat16()
    w = (torch.randn(3, 3, Cin, Cout, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cout, device=cuda_dev)
    wp = pack_fwd(w)
    outs = []
    for rev in (0, 1):
        y = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16)
        bits = torch.zeros(N * H * H * Cout // 8, device=cuda_dev, dtype=torch.uint8)
        # (zero-filled: at H = 256 no pool is fused and these stay unwritten -- uninitialised
        # memory of two allocations would differ)
        pooled = torch.zeros(N, H // 2, H // 2, Cout, device=cuda_dev, dtype=torch.bfloat16)
        codes = torch.zeros(N * (H // 2) ** 2 * Cout // 8, device=cuda_dev, dtype=torch.int32)
        d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, src1=ptr(x), wgt=ptr(wp), bias=ptr(b),
                 Cout=Cout, relu=1, dst1=ptr(y), relu_bits=ptr(bits), tile=tile, rev=rev)
        if H <= 128:
            d.update(pool_dst=ptr(pooled), pool_code=ptr(codes))
        assert C().conv_fwd_grid(d) > 0
        C().conv_fwd(d, stream())
        torch.cuda.synchronize()
        outs.append((y, bits, pooled, codes))
    for a, bb in zip(*outs):
        assert torch.equal(a, bb)
    ref = nhwc(F.relu(F.conv2d(nchw(x.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    assert rel_err(outs[1][0], ref) < 1e-2


def _relu_bits(x):
    """[P, C] 16-bit activation -> [P, C / 8] uint8, bit e of byte b = x[p, 8b + e] > 0."""
    P, Cc = x.shape[0], x.shape[-1]
    pos = (x.reshape(P, Cc // 8, 8).float() > 0).to(torch.int32)
    sh = torch.arange(8, device=x.device, dtype=torch.int32)
    return (pos << sh).sum(-1).to(torch.uint8).contiguous()


@pytest.mark.parametrize("N,H,Cy,bce,gs,splits", [(2, 128, 64, 0.0, 1.0, 5), (3, 64, 32, 0.5, 8.0, 3),
                                                  (4, 32, 64, 0.0, 1.0, 2), (5, 16, 32, 1.0, 2.0, 7),
                                                  (5, 16, 64, 0.0, 1.0, 3), (2, 16, 32, 0.0, 1.0, 3)])
def test_head_onload_matches_materialised_head_gradient(cuda_dev, N, H, Cy, bce, gs, splits):
    """Head-on-load (head_grad.h): the head input's data gradient and weight gradient
    forming dY = dlogit * w * (x > 0) from the probability, target and ReLU bits equal
    the same kernels reading the dY head_bwd materialises (same formula, same rounding:
    bit-identical), and head_bwd with dx = nullptr still reduces the Mask gradients."""
    torch.manual_seed(71)
    Cc = 32
    P = N * H * H
    x = F.relu(torch.randn(N, H, H, Cc, device=cuda_dev)).bfloat16()
    w = torch.randn(Cc, device=cuda_dev) * 0.3
    prob = torch.rand(P, device=cuda_dev) * 0.98 + 0.01
    t = (torch.rand(P, device=cuda_dev) > 0.6).bfloat16()
    sums = torch.stack([(t.float() * prob).sum(), t.float().sum(), prob.sum(), torch.zeros((), device=cuda_dev)])
    gsc = torch.full((1,), gs, device=cuda_dev)
    nb = C().head_blocks(P)
    part = torch.zeros(nb * (Cc + 1), device=cuda_dev)
    dy = torch.empty_like(x)
    ow0, ob0, ow1, ob1 = [torch.zeros(n, device=cuda_dev) for n in (Cc, 1, Cc, 1)]
    hb = lambda dx, ow, ob: C().generic("head_bwd", [ptr(x), ptr(w), ptr(prob), ptr(t), ptr(sums), dx, ptr(part),
                                                     ptr(ow), ptr(ob), ptr(gsc)], [P, Cc], [1.0 / P, bce, 1.0],
                                        stream())
    hb(ptr(dy), ow0, ob0)
    hb(0, ow1, ob1)
    bits = _relu_bits(x.reshape(P, Cc))
    hg = dict(hg_prob=ptr(prob), hg_t=ptr(t), hg_sums=ptr(sums), hg_w=ptr(w), hg_bits=ptr(bits), hg_gscale=ptr(gsc),
              hg_inv_total=1.0 / P, hg_bce_w=bce)
    # data gradient into a ReLU'd input (bit mask), as dgrad:conv9b
    a9 = torch.randn(N, H, H, Cy, device=cuda_dev).bfloat16()
    a9b = _relu_bits(a9.reshape(P, Cy))
    wt = (torch.randn(3, 3, Cy, Cc, device=cuda_dev) * 0.1).bfloat16()
    wp = pack_dgrad(wt)                          # kept alive: later allocations must not reuse it
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cc, src1=ptr(dy), wgt=ptr(wp), Cout=Cy,
             mask1=ptr(a9b), mask_bits=1)
    dx0, dx1 = torch.empty_like(a9), torch.full_like(a9, float("nan"))
    C().conv_fwd(dict(d, dst1=ptr(dx0)), stream())
    C().conv_fwd(dict(d, dst1=ptr(dx1), src1=ptr(x), **hg), stream())     # src1 unused: dY formed on load
    # weight + bias gradient (B = dY)
    a = F.relu(a9.float()).bfloat16()
    base = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=Cy, a1=ptr(a), Nc=Cc, bias_mode=1)
    g0, b0 = _wgrad(dict(base, b=ptr(dy)), splits, 9, Cy, Cy, Cc, 9 * Cy * Cc, bias_w=(splits, Cc))
    g1, b1 = _wgrad(dict(base, b=ptr(x), **hg), splits, 9, Cy, Cy, Cc, 9 * Cy * Cc, bias_w=(splits, Cc))
    torch.cuda.synchronize()
    # the materialised path itself against autograd (fp32 head, ReLU mask)
    pr = prob.clone().requires_grad_(True)
    tf = t.float()
    z = torch.log(pr / (1 - pr))
    zz = z.detach().requires_grad_(True)
    pz = torch.sigmoid(zz)
    loss = (-torch.log(2 * (tf * pz).sum() + 1) + torch.log(tf.sum() + pz.sum() + 1)
            + bce * F.binary_cross_entropy_with_logits(zz, tf, reduction="sum") / P) * gs
    (dlog,) = torch.autograd.grad(loss, [zz])
    ref_dy = dlog[:, None] * w[None, :] * (x.reshape(P, Cc).float() > 0)
    assert rel_err(dy.reshape(P, Cc), ref_dy) < 1e-2
    xr = torch.zeros(N, Cy, H, H, device=cuda_dev, requires_grad=True)
    yr = F.conv2d(xr, wt.float().permute(3, 2, 0, 1), padding=1)
    (gx,) = torch.autograd.grad(yr, xr, nchw(dy.float()))
    ref_dx = nhwc(gx) * (a9.float() > 0)
    e0, e1 = rel_err(dx0, ref_dx), rel_err(dx1, ref_dx)
    assert e0 < 1e-2 and e1 < 1e-2, (e0, e1)
    assert torch.equal(dx0, dx1)
    assert torch.equal(g0, g1) and torch.equal(b0, b1)
    assert torch.equal(ow0, ow1) and torch.equal(ob0, ob1)


def test_row_window_kernels_beyond_2gib(cuda_dev):
    """Row-window forward / data gradient / weight gradient on a 32-channel tensor of
    2.2 GB (image-relative 32-bit DMA offsets): equal to the same launches on the two
    batch halves (each below 2 GiB) -- bit for bit for the convs, to fp32 summation
    order for the weight gradient."""
    torch.manual_seed(7)
    N, H, Cc = 2112, 128, 32
    h = N // 2
    x = torch.randn(N, H, H, Cc, device=cuda_dev, dtype=torch.bfloat16)
    assert x.numel() * 2 > 2 ** 31
    w = (torch.randn(3, 3, Cc, Cc, device=cuda_dev) * 0.1).bfloat16()
    b = torch.randn(Cc, device=cuda_dev)
    wp = pack_fwd(w)
    out = torch.empty_like(x)
    base = dict(OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cc, wgt=ptr(wp), bias=ptr(b), Cout=Cc, relu=1)
    C().conv_fwd(dict(base, N=N, src1=ptr(x), dst1=ptr(out)), stream())
    assert C().conv_fwd_grid(dict(base, N=N, src1=ptr(x), dst1=ptr(out))) > 0
    ref = torch.empty_like(x)
    for k in range(2):
        C().conv_fwd(dict(base, N=h, src1=ptr(x[k * h:]), dst1=ptr(ref[k * h:])), stream())
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    del out, ref
    # weight gradient: a = x, b = dY (same shape)
    dy = torch.randn(N, H, H, Cc, device=cuda_dev, dtype=torch.bfloat16)
    kd = dict(QD=1, QH=H, QW=H, AD=1, AH=H, AW=H, KD=1, KH=3, KW=3, stride=1, pad=1, M1=Cc, M2=0, Nc=Cc,
              bias_mode=1, win=0)
    full, fb = _wgrad(dict(kd, N=N, a1=ptr(x), b=ptr(dy)), 64, 9, Cc, Cc, Cc, 9 * Cc * Cc, bias_w=(64, Cc))
    parts = [_wgrad(dict(kd, N=h, a1=ptr(x[k * h:]), b=ptr(dy[k * h:])), 32, 9, Cc, Cc, Cc, 9 * Cc * Cc,
                    bias_w=(32, Cc)) for k in range(2)]
    torch.cuda.synchronize()
    assert rel_err(full, parts[0][0] + parts[1][0]) < 1e-4
    assert rel_err(fb, parts[0][1] + parts[1][1]) < 1e-4


@pytest.mark.parametrize("N,C1,C2,Cout,drop", [(5, 256, 0, 512, 0.0), (8, 512, 0, 512, 0.2), (3, 64, 64, 128, 0.0),
                                              (4, 32, 0, 64, 0.0)])
def test_conv_img8_forward(cuda_dev, N, C1, C2, Cout, drop):
    """8x8 image-window kernel (tile 13, auto at 8x8): bias + ReLU (+ dropout, generic
    epilogue) + ReLU bits vs the fp32 reference; a partial last workgroup (N % 4); the
    dropout keep-mask equals the implicit-GEMM kernel's (tile 1 / 2)."""
    torch.manual_seed(51)
    dev = cuda_dev
    x = torch.randn(N, 8, 8, C1, device=dev).bfloat16()
    sk = torch.randn(N, 8, 8, C2, device=dev).bfloat16() if C2 else None
    w = (torch.randn(3, 3, C1 + C2, Cout, device=dev) * 0.05).bfloat16()
    b = torch.randn(Cout, device=dev) * 0.1
    assert C().conv_fwd_pick(dict(N=N, OH=8, OW=8, IH=8, IW=8, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=1,
                                  src2=1 if C2 else None, wgt=1, Cout=Cout, relu=1, dst1=1, drop_rate=drop)) == 13
    outs = {}
    for tile in (13, 2):
        y = torch.full((N, 8, 8, Cout), float("nan"), device=dev, dtype=torch.bfloat16)
        bits = torch.zeros(N, 8, 8, Cout // 8, device=dev, dtype=torch.uint8)
        wp = pack_fwd(w)
        C().conv_fwd(dict(N=N, OH=8, OW=8, IH=8, IW=8, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(x),
                          src2=ptr(sk) if C2 else None, wgt=ptr(wp), bias=ptr(b), Cout=Cout, relu=1,
                          drop_rate=drop, seed=7, salt=2, dst1=ptr(y), relu_bits=ptr(bits), tile=tile), stream())
        torch.cuda.synchronize()
        assert torch.equal(bits, _pack_bits(y))
        outs[tile] = y
    xin = torch.cat([x, sk], -1) if C2 else x
    ref = nhwc(F.relu(F.conv2d(nchw(xin.float()), w.float().permute(3, 2, 0, 1), b, padding=1)))
    y = outs[13]
    if drop:
        keep = outs[2].float() != 0
        assert torch.equal(keep, y.float() != 0) or (keep ^ (y.float() != 0)).float().mean() < 1e-3
        ref = ref * keep / (1 - drop)
    assert rel_err(y, ref) < 1e-2
    assert rel_err(y, outs[2]) < 1e-2


def test_conv_img8_dgrad_dual_dest_bit_masks(cuda_dev):
    """8x8 image-window data gradient: flipped weights, two destinations, ReLU bit masks
    and a dropout rescale on the second."""
    torch.manual_seed(52)
    dev = cuda_dev
    N, C1, C2, Co = 6, 256, 256, 512
    m1 = torch.randn(N, 8, 8, C1, device=dev).bfloat16()
    m2 = torch.randn(N, 8, 8, C2, device=dev).bfloat16()
    w = (torch.randn(3, 3, C1 + C2, Co, device=dev) * 0.05).bfloat16()
    dy = torch.randn(N, 8, 8, Co, device=dev).bfloat16()
    d1 = torch.empty(N, 8, 8, C1, device=dev, dtype=torch.bfloat16)
    d2 = torch.empty(N, 8, 8, C2, device=dev, dtype=torch.bfloat16)
    b1, b2, wd = _pack_bits(m1), _pack_bits(m2), pack_dgrad(w)      # (kept alive across the launch)
    d = dict(N=N, OH=8, OW=8, IH=8, IW=8, KH=3, KW=3, pad=1, C1=Co, src1=ptr(dy), wgt=ptr(wd),
             Cout=C1 + C2, D1=C1, dst1=ptr(d1), dst2=ptr(d2), mask1=ptr(b1), mask2=ptr(b2),
             mask_bits=3, mask_scale2=1.25)
    assert C().conv_fwd_pick(d) == 13
    C().conv_fwd(d, stream())
    xr = torch.zeros(N, C1 + C2, 8, 8, device=dev, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv2d(xr, w.float().permute(3, 2, 0, 1), padding=1), xr, nchw(dy.float()))
    g = nhwc(g)
    torch.cuda.synchronize()
    assert rel_err(d1, g[..., :C1] * (m1.float() > 0)) < 1e-2
    assert rel_err(d2, g[..., C1:] * (m2.float() > 0) * 1.25) < 1e-2


def test_conv_img8_norm_statistics(cuda_dev):
    """8x8 image window with the fused-normalisation epilogues (BatchNorm): the pre-norm
    forward's per-tile {sum z, sum z^2} rows and the dgrad-norm epilogue's masked gradient
    + {sum g, sum g z} rows reduce to the implicit-GEMM kernel's (tile 2) totals."""
    torch.manual_seed(53)
    dev, N, Ci, Co = cuda_dev, 6, 256, 512
    x = torch.randn(N, 8, 8, Ci, device=dev).bfloat16()
    w = (torch.randn(3, 3, Ci, Co, device=dev) * 0.05).bfloat16()
    b = torch.randn(Co, device=dev) * 0.1
    wp = pack_fwd(w)
    na, nc = torch.rand(Co, device=dev) + 0.5, torch.randn(Co, device=dev) * 0.1
    dy = torch.randn(N, 8, 8, Co, device=dev).bfloat16()
    w2 = (torch.randn(3, 3, Co, Co, device=dev) * 0.05).bfloat16()
    wd = pack_dgrad(w2)
    res = {}
    for tile in (13, 2):
        geo = dict(N=N, OH=8, OW=8, IH=8, IW=8, KH=3, KW=3, pad=1, tile=tile)
        df = dict(geo, C1=Ci, src1=ptr(x), wgt=ptr(wp), bias=ptr(b), Cout=Co, relu=0, stats=1, dst1=1)
        rows, _ = C().conv_stat_tiles(df)
        z = torch.empty(N, 8, 8, Co, device=dev, dtype=torch.bfloat16)
        st = torch.zeros(rows, 2, Co, device=dev)
        C().conv_fwd(dict(df, dst1=ptr(z), stats=ptr(st)), stream())
        dd = dict(geo, C1=Co, src1=ptr(dy), wgt=ptr(wd), Cout=Co, relu=0, stats=1, nz=ptr(z), na=ptr(na), nc=ptr(nc),
                  npix=64, dst1=1)
        rows2, _ = C().conv_stat_tiles(dd)
        g = torch.empty(N, 8, 8, Co, device=dev, dtype=torch.bfloat16)
        st2 = torch.zeros(rows2, 2, Co, device=dev)
        C().conv_fwd(dict(dd, dst1=ptr(g), stats=ptr(st2)), stream())
        torch.cuda.synchronize()
        res[tile] = (z, st.sum(0), g, st2.sum(0))
    (z0, s0, g0, t0), (z1, s1, g1, t1) = res[13], res[2]
    assert rel_err(z0, z1) < 1e-2 and rel_err(g0, g1) < 1e-2
    assert rel_err(s0, s1) < 1e-2 and rel_err(t0, t1) < 1e-2
    zf = z0.float().reshape(-1, Co)
    assert rel_err(s0[0], zf.sum(0)) < 1e-3 and rel_err(s0[1], (zf * zf).sum(0)) < 1e-3



@pytest.mark.parametrize("N,D,Ci,Co,tile", [(2, 16, 64, 32, 0), (1, 32, 128, 64, 0), (1, 64, 64, 32, 0),
                                           (2, 16, 64, 32, 8), (1, 8, 256, 128, 0)])
def test_tconv3d_fwd_window(cuda_dev, N, D, Ci, Co, tile):
    """2x2x2 stride-2 transposed conv forward (3D model): the transposed-conv window kernel
    (eight taps, two per wave; coarse rows 16..128 wide) against fp32 ATen, and equal to the
    implicit-GEMM shuffle path (tile 8) within rounding."""
    torch.manual_seed(D + Ci)
    x = F.relu(torch.randn(N, D, D, D, Ci, device=cuda_dev)).bfloat16()
    k = (torch.randn(2, 2, 2, Co, Ci, device=cuda_dev) * 0.1).bfloat16()   # (kd, kh, kw, Cout, Cin)
    b = torch.randn(Co, device=cuda_dev)
    out = torch.empty(N, 2 * D, 2 * D, 2 * D, Co, device=cuda_dev, dtype=torch.bfloat16)
    C().conv_fwd(dict(N=N, OD=D, OH=D, OW=D, ID=D, IH=D, IW=D, C1=Ci, src1=ptr(x),
                      wgt=ptr(pad64(k.reshape(8 * Co, Ci))), bias=ptr(b), Cout=8 * Co, shuffle=3, dst1=ptr(out),
                      tile=tile), stream())
    wt = k.float().permute(4, 3, 0, 1, 2)     # (Cin, Cout, kd, kh, kw)
    ref = ndhwc(F.conv_transpose3d(ncdhw(x.float()), wt, b, stride=2))
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("N,D,H,C1,C2,Cout,splits", [(1, 4, 32, 32, 0, 32, 3), (2, 3, 64, 32, 32, 32, 5),
                                                      (1, 3, 128, 32, 0, 32, 4), (1, 4, 128, 32, 32, 64, 7),
                                                      (3, 1, 128, 32, 0, 32, 5), (2, 1, 64, 64, 0, 32, 3),
                                                      (2, 1, 32, 32, 32, 64, 4), (1, 1, 256, 32, 0, 32, 6)])
def test_wgrad_window_wave_pair(cuda_dev, N, D, H, C1, C2, Cout, splits):
    """Wave-pair partials (pair=1: each wave one 16-channel half of its 32-channel output
    block, three workgroups per CU) against the fp32 reference: 3D (D > 1) and 2D rows,
    concat sources, segmented 256-wide rows."""
    torch.manual_seed(N + D + H + C1 + C2 + 11)
    d3 = D > 1
    shp = (N, D, H, H) if d3 else (N, H, H)
    a = F.relu(torch.randn(*shp, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(*shp, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(*shp, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    T = 27 if d3 else 9
    d = dict(N=N, QD=D, QH=H, QW=H, AD=D, AH=H, AW=H, KD=3 if d3 else 1, KH=3, KW=3, pad=1, M1=C1, M2=C2,
             a1=ptr(a), a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1, pair=1)
    gw, gb = _wgrad(d, splits, T, Mt, Mt, Cout, T * Mt * Cout, bias_w=(splits, Cout))
    conv, to_nc = (F.conv3d, ncdhw) if d3 else (F.conv2d, nchw)
    inp = to_nc(a.float()) if not C2 else torch.cat([to_nc(a.float()), to_nc(b2.float())], 1)
    ks = (3, 3, 3) if d3 else (3, 3)
    w = torch.zeros(Cout, Mt, *ks, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(conv(inp, w, bb, padding=1), [w, bb], to_nc(dy.float()))
    perm = (2, 3, 4, 1, 0) if d3 else (2, 3, 1, 0)
    assert rel_err(gw, gwr.permute(*perm).reshape(-1)) < 2e-3
    assert rel_err(gb, gbr) < 2e-3


@pytest.mark.parametrize("N,D,H,C1,C2,Cout,splits", [(2, 1, 128, 32, 0, 32, 7), (3, 1, 128, 32, 32, 64, 5),
                                                      (1, 8, 128, 32, 0, 32, 6), (1, 6, 128, 32, 32, 32, 4),
                                                      (2, 1, 128, 64, 0, 32, 64)])
def test_wgrad_window_prefetch_equals_dma(cuda_dev, N, D, H, C1, C2, Cout, splits):
    """Prefetching 128-wide window weight gradient (pf=1: the next window's new halo rows and
    dY in registers under the current window's MFMAs) equals the LDS-DMA window kernel bit
    for bit (same images, fragment reads, MFMA order, reduction); 2D and 3D rows, concat
    sources, windows at image / slice starts (no carry) and split ranges that start inside
    an image."""
    torch.manual_seed(N + D + C1 + C2 + splits)
    d3 = D > 1
    shp = (N, D, H, H) if d3 else (N, H, H)
    a = F.relu(torch.randn(*shp, C1, device=cuda_dev)).bfloat16()
    b2 = F.relu(torch.randn(*shp, max(C2, 1), device=cuda_dev)).bfloat16()
    dy = torch.randn(*shp, Cout, device=cuda_dev).bfloat16()
    Mt = C1 + C2
    T = 27 if d3 else 9
    d = dict(N=N, QD=D, QH=H, QW=H, AD=D, AH=H, AW=H, KD=3 if d3 else 1, KH=3, KW=3, pad=1, M1=C1, M2=C2,
             a1=ptr(a), a2=ptr(b2) if C2 else None, b=ptr(dy), Nc=Cout, bias_mode=1)
    out = []
    for pf in (0, 1):
        gw, gb = _wgrad(dict(d, pf=pf), splits, T, Mt, Mt, Cout, T * Mt * Cout, bias_w=(splits, Cout))
        out.append((gw, gb))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    conv, to_nc = (F.conv3d, ncdhw) if d3 else (F.conv2d, nchw)
    inp = to_nc(a.float()) if not C2 else torch.cat([to_nc(a.float()), to_nc(b2.float())], 1)
    ks = (3, 3, 3) if d3 else (3, 3)
    w = torch.zeros(Cout, Mt, *ks, device=cuda_dev, requires_grad=True)
    gwr, = torch.autograd.grad(conv(inp, w, padding=1), [w], to_nc(dy.float()))
    perm = (2, 3, 4, 1, 0) if d3 else (2, 3, 1, 0)
    assert rel_err(out[1][0], gwr.permute(*perm).reshape(-1)) < 2e-3
