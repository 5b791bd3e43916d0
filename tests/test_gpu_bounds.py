"""Bounds sentinels for the prefetching / persistent window kernels (round-5 verdict: the
3D first-layer window once read past the last volume -- a caching-allocator tensor has
slack after it, so an ordinary test cannot see such a read).  Every input operand is
carved out of a larger buffer whose head and tail are NaN (16-bit / fp32 operands) or
0xFF bytes (bit masks, codes), and the launch runs the shapes whose last window /
workgroup / volume touches the tensor end: the outputs must be finite and equal to the
run on ordinary allocations.  Kernels: conv_win_pf (persistent level-1 window, forward
and data gradient, also segmented rows), conv_win_pfu (persistent tconv-on-load window),
conv_win_cp (chunk-pipelined 64-channel window), the 3D first-layer window, and the fused
data + weight gradient conv_dw in all its operand sources (XF 0 / 2 / 3 / 4) with the
halo-row carry."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, _pack_bits, pack_dgrad, pack_fwd, pad64, ptr, stream

pytestmark = pytest.mark.gpu
PAD = 1 << 16          # guard elements on each side


def guarded(t):
    """A copy of `t` in the middle of a buffer whose PAD elements before and after it are
    poison (NaN for float types, all-ones bits for integer types)."""
    flat = t.reshape(-1)
    if t.dtype.is_floating_point:
        buf = torch.full((flat.numel() + 2 * PAD,), float("nan"), dtype=t.dtype, device=t.device)
    else:
        buf = torch.full((flat.numel() + 2 * PAD,), 255 if t.dtype == torch.uint8 else -1, dtype=t.dtype,
                         device=t.device)
    buf[PAD:PAD + flat.numel()] = flat
    return buf[PAD:PAD + flat.numel()].view(t.shape)


def _run(d, outs):
    """Launch conv dict `d` (tensors in place of pointers) with fresh NaN-filled outputs."""
    res = {k: torch.full_like(v, float("nan")) if v.dtype.is_floating_point else torch.zeros_like(v)
           for k, v in outs.items()}
    q = {k: (ptr(v) if isinstance(v, torch.Tensor) else v) for k, v in d.items()}
    q.update({k: ptr(v) for k, v in res.items()})
    C().conv_fwd(q, stream())
    torch.cuda.synchronize()
    return res


def _check(d, outs, inputs):
    """Same launch on ordinary and on guarded copies of the `inputs` keys of `d`."""
    ref = _run(d, outs)
    g = dict(d)
    keep = [guarded(d[k]) for k in inputs]
    g.update(dict(zip(inputs, keep)))
    got = _run(g, outs)
    for k in outs:
        if outs[k].dtype.is_floating_point:
            assert torch.isfinite(got[k].float()).all(), k
        assert torch.equal(got[k], ref[k]), k


@pytest.mark.parametrize("N,W,pf,rev", [(3, 128, 5, 0), (3, 128, 5, 1), (1, 512, 3, 1)])
def test_win_pf_forward_bounds(cuda_dev, N, W, pf, rev):
    torch.manual_seed(1)
    H = W if W <= 128 else 16
    x = F.relu(torch.randn(N, H, W, 32, device=cuda_dev)).bfloat16()
    wp = pack_fwd((torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16())
    b = torch.randn(32, device=cuda_dev) * 0.1
    d = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=x, wgt=wp, bias=b, Cout=32, relu=1,
             win_pf=pf, rev=rev)
    outs = dict(dst1=torch.empty(N, H, W, 32, device=cuda_dev, dtype=torch.bfloat16))
    _check(d, outs, ["src1", "wgt", "bias"])


@pytest.mark.parametrize("N,pf,rev", [(3, 3, 1), (2, 16, 0)])
def test_win_pf_dgrad_route_bounds(cuda_dev, N, pf, rev):
    torch.manual_seed(2)
    H = 128
    y = F.relu(torch.randn(N, H, H, 32, device=cuda_dev)).bfloat16()
    pooled = torch.empty(N, H // 2, H // 2, 32, device=cuda_dev, dtype=torch.bfloat16)
    codes = torch.zeros(N * (H // 2) ** 2 * 4, device=cuda_dev, dtype=torch.int32)
    C().generic("pool_fwd", [ptr(y), ptr(pooled), ptr(codes)], [N, 1, H, H, 32, 0], [], stream())
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32,
             src1=torch.randn(N, H, H, 32, device=cuda_dev).bfloat16(),
             wgt=pack_dgrad((torch.randn(3, 3, 32, 32, device=cuda_dev) * 0.1).bfloat16()), Cout=32,
             mask1=_pack_bits(y), mask_bits=1, route_gy=torch.randn(N, H // 2, H // 2, 32, device=cuda_dev).bfloat16(),
             pool_code=codes, win_pf=pf, rev=rev)
    outs = dict(dst1=torch.empty(N, H, H, 32, device=cuda_dev, dtype=torch.bfloat16))
    _check(d, outs, ["src1", "mask1", "route_gy", "pool_code"])


@pytest.mark.parametrize("N,K,pf", [(3, 32, 5), (2, 64, 8)])
def test_win_pfu_tconv_onload_bounds(cuda_dev, N, K, pf):
    torch.manual_seed(3)
    H = 64
    F2 = 2 * H
    b = F.relu(torch.randn(N, H, H, K, device=cuda_dev)).bfloat16()
    skip = torch.randn(N, F2, F2, 32, device=cuda_dev).bfloat16()
    wt = pad64((torch.randn(4 * 32, K, device=cuda_dev) * 0.1).bfloat16())
    wa = pad64((torch.randn(32, 9 * 64, device=cuda_dev) * 0.1).bfloat16())
    d = dict(N=N, OH=F2, OW=F2, IH=F2, IW=F2, KH=3, KW=3, pad=1, C1=32, C2=32, src1=b, src2=skip, wgt=wa,
             bias=torch.randn(32, device=cuda_dev) * 0.1, Cout=32, relu=1, ut_x=b, ut_w=wt,
             ut_b=torch.randn(32, device=cuda_dev) * 0.1, ut_C=K, ut_kpad=wt.shape[1], win_pf=pf)
    outs = dict(dst1=torch.empty(N, F2, F2, 32, device=cuda_dev, dtype=torch.bfloat16))
    # (src1 and ut_x are the same tensor: guard it once, as ut_x)
    ref = _run(d, outs)
    gb = guarded(b)
    g = dict(d, src1=gb, ut_x=gb, src2=guarded(skip), ut_w=guarded(wt), wgt=guarded(wa))
    got = _run(g, outs)
    assert torch.isfinite(got["dst1"].float()).all() and torch.equal(got["dst1"], ref["dst1"])


@pytest.mark.parametrize("N,H,C1,C2,Cout", [(2, 64, 64, 64, 64), (3, 64, 128, 0, 64)])
def test_win_cp_bounds(cuda_dev, N, H, C1, C2, Cout):
    torch.manual_seed(4)
    d = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2,
             src1=F.relu(torch.randn(N, H, H, C1, device=cuda_dev)).bfloat16(),
             wgt=pack_fwd((torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.05).bfloat16()),
             bias=torch.randn(Cout, device=cuda_dev) * 0.1, Cout=Cout, relu=1, win_cp=1)
    inputs = ["src1", "wgt", "bias"]
    if C2:
        d["src2"] = F.relu(torch.randn(N, H, H, C2, device=cuda_dev)).bfloat16()
        inputs.append("src2")
    outs = dict(dst1=torch.empty(N, H, H, Cout, device=cuda_dev, dtype=torch.bfloat16))
    _check(d, outs, inputs)


@pytest.mark.parametrize("N,D,H,Cin", [(1, 5, 128, 8), (2, 3, 64, 4)])
def test_conv3d_first_layer_window_bounds(cuda_dev, N, D, H, Cin):
    """The last volume's last depth slice: its d + 1 taps must read the zero padding, not
    the bytes after the tensor (the run-P fault of round 5)."""
    torch.manual_seed(5)
    Co = 32
    w = (torch.randn(3, 3, 3, Cin, Co, device=cuda_dev) * 0.1).bfloat16()
    d = dict(N=N, OD=D, OH=H, OW=H, ID=D, IH=H, IW=H, KD=3, KH=3, KW=3, pad=1, C1=Cin,
             src1=torch.randn(N, D, H, H, Cin, device=cuda_dev).bfloat16(),
             wgt=pad64(w.permute(4, 0, 1, 2, 3).reshape(Co, -1)), bias=torch.randn(Co, device=cuda_dev), Cout=Co,
             relu=1, tile=9)
    outs = dict(dst1=torch.empty(N, D, H, H, Co, device=cuda_dev, dtype=torch.bfloat16))
    _check(d, outs, ["src1", "wgt", "bias"])


@pytest.mark.parametrize("xf,N,nsplit,W", [(0, 3, 7, 128), (2, 3, 7, 128), (3, 2, 5, 128), (4, 3, 96, 128),
                                           (0, 2, 512, 128), (0, 1, 5, 512)])
def test_conv_dw_bounds(cuda_dev, xf, N, nsplit, W):
    """The fused data + weight gradient: halo rows of the first / last image, the carried
    halo rows of consecutive windows, the last workgroup's window range (W = 512: the
    segmented rows' neighbour-segment halo columns)."""
    torch.manual_seed(6 + xf)
    H = 128 if W == 128 else 32
    dev = cuda_dev
    P = N * H * W
    x = F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()
    d = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32,
             src1=torch.randn(N, H, W, 32, device=dev).bfloat16(),
             wgt=pack_dgrad((torch.randn(3, 3, 32, 32, device=dev) * 0.1).bfloat16()), Cout=32, relu=0, fw_x=x,
             fw_Cx=32, fw_nsplit=nsplit)
    inputs = ["src1", "wgt", "fw_x"]
    outs = dict(dst1=torch.empty(N, H, W, 32, device=dev, dtype=torch.bfloat16),
                fw_slab=torch.empty(nsplit, 9, 32, 32, device=dev), fw_bias_slab=torch.empty(nsplit, 32, device=dev))
    if xf == 0 or xf == 4:
        d.update(mask1=_pack_bits(F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16()), mask_bits=1)
        inputs.append("mask1")
    else:
        rows = N if xf == 3 else 1
        d.update(nz=torch.randn(N, H, W, 32, device=dev).bfloat16(), na=0.5 + torch.rand(rows, 32, device=dev),
                 nc=0.2 * torch.randn(rows, 32, device=dev), ncs=32 if rows > 1 else 0, npix=H * W)
        inputs += ["nz", "na", "nc"]
        outs["stats"] = torch.empty(N * H // 2, 2, 32, device=dev)
    if xf in (2, 3):
        rows = N if xf == 3 else 1
        d.update(xform=2, xz=torch.randn(N, H, W, 32, device=dev).bfloat16(), xa=0.5 + torch.rand(rows, 32, device=dev),
                 xb=0.2 * torch.randn(rows, 32, device=dev), xc=0.1 * torch.randn(rows, 32, device=dev),
                 xcs=32 if rows > 1 else 0)
        inputs += ["xz", "xa", "xb", "xc"]
    if xf in (3, 4):
        pr = torch.rand(P, device=dev) * 0.98 + 0.01
        t = (torch.rand(P, device=dev) > 0.7).bfloat16()
        d.update(hg_prob=pr, hg_t=t, hg_sums=torch.tensor([50.0, 70.0, 90.0, 0.0], device=dev),
                 hg_w=0.3 * torch.randn(32, device=dev), hg_inv_total=1.0 / P, hg_bce_w=0.5)
        inputs += ["hg_prob", "hg_t", "hg_w"]
        if xf == 4:
            d["hg_bits"] = _pack_bits(F.relu(torch.randn(N, H, W, 32, device=dev)).bfloat16())
            inputs.append("hg_bits")
        else:
            d.update(src1=d["xz"], hg_fa=0.5 + torch.rand(N, 32, device=dev), hg_fc=0.2 * torch.randn(N, 32, device=dev))
            inputs = [k for k in inputs if k not in ("src1", "xz")] + ["hg_fa", "hg_fc"]
    if xf == 3:
        # (src1 and xz are the same z: guard it once)
        ref = _run(d, outs)
        gz = guarded(d["xz"])
        g = dict(d, src1=gz, xz=gz, **{k: guarded(d[k]) for k in inputs})
        got = _run(g, outs)
        for k in outs:
            assert torch.isfinite(got[k].float()).all(), k
            assert torch.equal(got[k], ref[k]), k
        return
    _check(d, outs, inputs)
