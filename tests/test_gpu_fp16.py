"""fp16 build of the kernels (``dtype=1``: namespace unet_f16, v_mfma_f32_16x16x32_f16)
against fp32 PyTorch references on fp16-rounded inputs, plus the fp16 training step
(GroupNorm, dynamic loss scaling) against the fp32 ATen step.

Same kernel sources as the bf16 tests (tests/test_gpu_kernels.py); fp16's 10-bit
mantissa gives tighter tolerances than bf16.
"""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import C, nchw, nhwc, pack_fwd, ptr, rel_err, stream

pytestmark = pytest.mark.gpu
H16 = torch.float16
FP16 = 1


@pytest.mark.parametrize("N,H,C1,C2,Cout,tile", [(2, 64, 32, 0, 32, 6), (3, 32, 64, 64, 64, 6), (2, 16, 64, 0, 64, 0),
                                                 (2, 8, 64, 0, 128, 0)])
def test_fp16_conv_fwd(cuda_dev, N, H, C1, C2, Cout, tile):
    torch.manual_seed(N + H + C1)
    a = torch.randn(N, H, H, C1, device=cuda_dev).half()
    b2 = torch.randn(N, H, H, max(C2, 1), device=cuda_dev).half()
    w = (torch.randn(3, 3, C1 + C2, Cout, device=cuda_dev) * 0.08).half()
    bias = torch.randn(Cout, device=cuda_dev) * 0.1
    out = torch.empty(N, H, H, Cout, device=cuda_dev, dtype=H16)
    C().conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(a),
                      src2=ptr(b2) if C2 else None, wgt=ptr(pack_fwd(w)), bias=ptr(bias), Cout=Cout, relu=1,
                      dst1=ptr(out), tile=tile), stream(), dtype=FP16)
    xin = nchw(a.float()) if not C2 else torch.cat([nchw(a.float()), nchw(b2.float())], 1)
    ref = nhwc(F.relu(F.conv2d(xin, w.float().permute(3, 2, 0, 1), bias, padding=1)))
    assert rel_err(out, ref) < 2e-3


@pytest.mark.parametrize("N,H,Cin,Cout,splits,win", [(3, 64, 32, 32, 5, 0), (2, 32, 64, 64, 3, 0),
                                                     (2, 16, 64, 128, 2, -1)])
def test_fp16_wgrad(cuda_dev, N, H, Cin, Cout, splits, win):
    from test_gpu_kernels import _wgrad
    torch.manual_seed(N + H + Cin)
    a = F.relu(torch.randn(N, H, H, Cin, device=cuda_dev)).half()
    dy = torch.randn(N, H, H, Cout, device=cuda_dev).half()
    d = dict(N=N, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=Cin, a1=ptr(a), b=ptr(dy), Nc=Cout,
             bias_mode=1, win=win)
    dev = torch.device("cuda")
    slab = torch.zeros(splits * 9 * Cin * Cout, device=dev)
    bslab = torch.zeros(splits * 8 * max(Cin, Cout), device=dev)
    C().wgrad(dict(d, splits=splits, slab=ptr(slab), bias_slab=ptr(bslab)), stream(), dtype=FP16)
    gw = slab.view(splits, -1).sum(0)
    gb = bslab[:splits * Cout].view(splits, Cout).sum(0)
    w = torch.zeros(Cout, Cin, 3, 3, device=cuda_dev, requires_grad=True)
    bb = torch.zeros(Cout, device=cuda_dev, requires_grad=True)
    gwr, gbr = torch.autograd.grad(F.conv2d(nchw(a.float()), w, bb, padding=1), [w, bb], nchw(dy.float()))
    assert rel_err(gw, gwr.permute(2, 3, 1, 0).reshape(-1)) < 1e-3
    assert rel_err(gb, gbr) < 1e-3


def test_fp16_pool_and_head_with_device_loss_scale(cuda_dev):
    torch.manual_seed(3)
    N, H, Cc = 2, 16, 32
    x = F.relu(torch.randn(N, H, H, Cc, device=cuda_dev)).half()
    y = torch.empty(N, H // 2, H // 2, Cc, device=cuda_dev, dtype=H16)
    C().generic("pool_fwd", [ptr(x), ptr(y)], [N, 1, H, H, Cc, 0], [], stream(), dtype=FP16)
    assert (y.float() - nhwc(F.max_pool2d(nchw(x.float()), 2))).abs().max().item() == 0

    P = 4096
    xh = F.relu(torch.randn(P, Cc, device=cuda_dev)).half()
    w = torch.randn(Cc, device=cuda_dev) * 0.3
    b = torch.randn(1, device=cuda_dev)
    t = (torch.rand(P, device=cuda_dev) > 0.7).half()
    prob = torch.empty(P, device=cuda_dev)
    nb = C().head_blocks(P)
    part = torch.empty(nb * (Cc + 1) + 4 * nb, device=cuda_dev)
    sums = torch.empty(4, device=cuda_dev)
    C().generic("head_fwd", [ptr(xh), ptr(w), ptr(b), ptr(t), ptr(prob), ptr(part), ptr(sums)], [P, Cc], [],
                stream(), dtype=FP16)
    xr = xh.float().requires_grad_(True)
    z = xr @ w + b
    p = torch.sigmoid(z)
    tf = t.float()
    I, St, Sp = (tf * p).sum(), tf.sum(), p.sum()
    assert rel_err(prob, p) < 1e-4
    loss = -torch.log(2 * I + 1) + torch.log(St + Sp + 1)
    (gx,) = torch.autograd.grad(loss, [xr])
    scale = torch.tensor([4096.0], device=cuda_dev)    # read from device memory, floats[2] ignored
    dx = torch.empty_like(xh)
    ow = torch.empty(Cc, device=cuda_dev)
    ob = torch.empty(1, device=cuda_dev)
    C().generic("head_bwd", [ptr(xh), ptr(w), ptr(prob), ptr(t), ptr(sums), ptr(dx), ptr(part), ptr(ow),
                             ptr(ob), ptr(scale)], [P, Cc], [1.0 / P, 0.0, 1.0], stream(), dtype=FP16)
    assert rel_err(dx.float() / 4096.0, gx * (xh.float() > 0)) < 2e-3


def test_fp16_groupnorm_step_matches_fp32(cuda_dev):
    """Native fp16 + GroupNorm training step with loss scale 2^12 vs the fp32 ATen
    step: unscaled gradients agree per tensor."""
    from test_gpu_model import _cos, _setup
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=4, img_size=64, in_channels=4, norm="group",
                                              dtype="fp16")
    assert nb.engine.dtype == "fp16"
    scale = 4096.0
    nb.fwd_bwd(x, y, seed=77, grad_scale=scale)
    tb.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    assert torch.isfinite(fn.grad).all()
    g = fn.grad / scale
    sn, st = nb.sums().cpu(), tb.sums().cpu()
    assert torch.allclose(sn[:3], st[:3], rtol=2e-2, atol=1.0), (sn, st)
    for name, shape, off, n in fn.entries:
        gt = ft.grad[off:off + n]
        if gt.norm() < 1e-6:
            continue
        c = _cos(g[off:off + n], gt)
        assert c > (0.95 if name.endswith("/bias") else 0.98), (name, c)
    assert _cos(g, ft.grad) > 0.99


def test_fp16_training_with_dynamic_loss_scale(cuda_dev):
    """A few fp16 steps through the native Adam with the dynamic scaler: loss falls,
    no step is lost to overflow at the initial scale for this config."""
    from test_gpu_model import _setup
    from unet_distributed_amd.runtime.amp import LossScaler
    from unet_distributed_amd.runtime.optim import TFAdam
    from unet_distributed_amd.runtime.trainer import _NativeOpt
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=8, img_size=64, in_channels=4, norm="group",
                                              dtype="fp16", learning_rate=1e-3)
    nb.engine.repack()
    opt = TFAdam(fn, cfg, native=_NativeOpt(nb))
    sc = LossScaler("fp16")
    losses = []
    for i in range(20):
        s0 = sc.scale
        nb.fwd_bwd(x, y, seed=i, grad_scale=s0)
        if sc.update(fn.grad):
            opt.step(grad_scale=1.0 / s0)
        s = nb.sums().cpu()
        losses.append((-torch.log(2 * s[0] + 1) + torch.log(s[1] + s[2] + 1)).item())
    assert sc.skipped <= 2, sc.state_dict()
    assert losses[-1] < 0.8 * losses[0], losses
