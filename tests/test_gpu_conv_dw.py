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
