"""Per-layer oracle at the benched shape (per-GPU batch 1024, 128x128x4, bf16): one native
training step, then every conv layer whose operands the plan materialises is recomputed
from the captured tensors in fp32 (shifted-tap GEMMs on rocBLAS, no MIOpen): forward
outputs (first 64 images) and weight gradients over the whole batch -- the split-K sizing
(`wg_target`), window choices and 2 GiB chunking of the bench shape, which the whole-step
ATen parity (B <= 256) never reaches.  Dropout off (the oracle has no mask stream); the
kernels and plan are otherwise the benched ones."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_model import _setup

pytestmark = pytest.mark.gpu
NS = 64                      # images of the forward check


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def _taps(x):
    """3x3 'same' taps of NHWC x as [(dh, dw, [P, C] shifted copy)]."""
    N, H, W, C = x.shape
    xp = F.pad(x, (0, 0, 1, 1, 1, 1))
    for dh in range(3):
        for dw in range(3):
            yield dh, dw, xp[:, dh:dh + H, dw:dw + W, :].reshape(-1, C)


@pytest.fixture(scope="module")
def stepped(cuda_dev):
    spec, cfg, x, y, fn, nb, ft, tb = _setup(cuda_dev, batch_size=1024, img_size=128, in_channels=4, dropout=0.0)
    nb.fwd_bwd(x, y, seed=11)
    torch.cuda.synchronize()
    return spec, fn, nb.engine


def _inputs(e, spec, name):
    """The conv's input as an NHWC fp32 tensor (u first, then the skip), or None when the
    plan does not materialise it (a transposed conv formed on load)."""
    src1, up1, skip = e.inputs[name]
    if up1 != 1 or src1 not in e.bufs or src1 in getattr(e, "_ut_onload", {}).values():
        return None
    if name in getattr(e, "_ut_onload", {}):
        return None
    parts = [e.bufs[src1]] + ([e.bufs[skip]] if skip else [])
    return parts


def _relu_mask(e, name, n):
    """[n, H, W, C] bool: the ReLU bits the forward stored for `name` (first n images)."""
    bits = e.relu_bits[name]
    C = e.tinfo[name][1]
    per = bits.numel() // e.B
    v = bits[:n * per].to(torch.int32)
    m = (v.unsqueeze(-1) >> torch.arange(8, device=v.device, dtype=torch.int32)) & 1
    return m.reshape(n, -1, C).bool().reshape(n, 128, 128, C)


def test_bench_shape_forward_per_layer(stepped):
    spec, fn, e = stepped
    checked = 0
    for l in spec.layers:
        if l.kind != "conv":
            continue
        parts = _inputs(e, spec, l.name)
        if parts is None:
            continue
        xin = torch.cat([p[:NS].float() for p in parts], -1)
        w = fn.view(fn.master, l.name + "/kernel").bfloat16().float()          # [3, 3, Cin, Cout]
        b = fn.view(fn.master, l.name + "/bias").float()
        Cin = w.shape[2]
        xin = xin[..., :Cin] if xin.shape[-1] > Cin else xin
        if xin.shape[-1] < Cin:      # first layer: channel-padded input buffer
            xin = F.pad(xin, (0, Cin - xin.shape[-1]))
        out = torch.zeros(xin.shape[0] * xin.shape[1] * xin.shape[2], w.shape[3], device=xin.device)
        for dh, dw, xs in _taps(xin):
            out += xs @ w[dh, dw]
        ref = F.relu(out + b).reshape(*xin.shape[:3], -1)
        if l.name == e.head_in and e.fusions.get("head_wsum"):
            # (head_wsum: the head input is not stored -- its ReLU bits and the head's
            # probabilities are what the step keeps)
            mism = (_relu_mask(e, l.name, NS) != (ref > 0)).float().mean().item()
            assert mism < 1e-3, (l.name, mism)
            hw = fn.view(fn.master, "Mask/kernel").float().reshape(-1)
            hb = fn.view(fn.master, "Mask/bias").float()
            pref = torch.sigmoid(ref.bfloat16().float() @ hw + hb)
            assert _rel(e.prob.view(e.B, -1)[:NS].reshape(pref.shape), pref) < 2e-2
            checked += 1
            continue
        got = e.bufs[l.name][:NS].float()
        err = _rel(got, ref)
        assert err < 2e-2, (l.name, err)
        checked += 1
    assert checked >= 12


def test_bench_shape_weight_gradients_per_layer(stepped):
    spec, fn, e = stepped
    checked = []
    for l in spec.layers:
        if l.kind != "conv" or ("d:" + l.name) not in e.bufs:
            continue
        parts = _inputs(e, spec, l.name)
        if parts is None:
            continue
        g = fn.view(fn.grad, l.name + "/kernel").float()                       # [3, 3, Cin, Cout]
        Cin, Cout = g.shape[2], g.shape[3]
        dy = e.bufs["d:" + l.name].float().reshape(-1, Cout)
        xin = torch.cat([p.float() for p in parts], -1)
        if xin.shape[-1] < Cin:
            xin = F.pad(xin, (0, Cin - xin.shape[-1]))
        ref = torch.zeros_like(g)
        for dh, dw, xs in _taps(xin[..., :Cin]):
            ref[dh, dw] = xs.t() @ dy
        err = _rel(g, ref)
        assert err < 2e-2, (l.name, err)
        gb = fn.view(fn.grad, l.name + "/bias").float()
        assert _rel(gb, dy.sum(0)) < 2e-2, l.name
        checked.append(l.name)
        del xin, dy
    print("bench-shape weight gradients checked:", checked)
    assert len(checked) >= 8


def _dgrad(dy, w):
    """Data gradient of a 3x3 'same' conv: dX[q] = sum_tap dY[q - tap + 1] W[tap]^T
    (shifted-tap GEMMs on the padded dY, fp32)."""
    N, H, W, Co = dy.shape
    dyp = F.pad(dy, (0, 0, 1, 1, 1, 1))
    out = torch.zeros(N * H * W, w.shape[2], device=dy.device)
    for dh in range(3):
        for dw in range(3):
            out += dyp[:, 2 - dh:2 - dh + H, 2 - dw:2 - dw + W, :].reshape(-1, Co) @ w[dh, dw].t()
    return out.reshape(N, H, W, -1)


def test_bench_shape_data_gradients(stepped):
    """Data gradients at the bench shape (first NS images; a conv's data gradient is per
    image): conv1b's (the fused data + weight gradient, conv_dw.hip, in two batch halves),
    conv5b's (8x8 image window), conv9b's (its dY formed on load from the head: conv_dw
    XF 4) and conv9a's skip half (deferred, with the max-pool backward of pool1 routed in
    its epilogue)."""
    spec, fn, e = stepped
    b = e.bufs
    kern = lambda n: fn.view(fn.master, n + "/kernel").bfloat16().float()
    # conv1b -> d:conv1a, conv5b -> d:conv5a: masked by the source activation
    for lname, src in (("conv1b", "conv1a"), ("conv5b", "conv5a")):
        ref = _dgrad(b["d:" + lname][:NS].float(), kern(lname)) * (b[src][:NS].float() > 0)
        err = _rel(b["d:" + src][:NS].float(), ref)
        assert err < 2e-2, (lname, err)
    # conv9b: dY = dlogit w (y > 0) from the head's probability / target / loss sums
    P = e.npix(1)
    pr = e.prob.view(e.B, -1)[:NS].float()
    t = e.target.view(e.B, -1)[:NS].float()
    I, St, Sp = [v.item() for v in e.sums[:3]]
    dl = (-2.0 * t / (2 * I + 1) + 1.0 / (St + Sp + 1)) * pr * (1 - pr) + e.bce_weight * (pr - t) / P
    hw = fn.view(fn.master, "Mask/kernel").float().reshape(-1)
    pos9b = _relu_mask(e, "conv9b", NS) if e.fusions.get("head_wsum") else b["conv9b"][:NS].float() > 0
    dy9b = dl.reshape(NS, 128, 128, 1) * hw * pos9b
    ref = _dgrad(dy9b, kern("conv9b")) * (b["conv9a"][:NS].float() > 0)
    err = _rel(b["d:conv9a"][:NS].float(), ref)
    assert err < 2e-2, ("conv9b", err)
    # conv9a skip half: masked skip gradient + pool1's gradient routed to its first argmax
    w9a = kern("conv9a")
    cu = w9a.shape[2] - b["conv1b"].shape[-1]
    skip_g = _dgrad(b["d:conv9a"][:NS].float(), w9a[:, :, cu:, :])
    y1b = b["conv1b"][:NS].float()
    win = y1b.reshape(NS, 64, 2, 64, 2, 32).permute(0, 1, 3, 5, 2, 4).reshape(NS, 64, 64, 32, 4)
    mx, am = win.max(-1)
    route = torch.zeros_like(win)
    route.scatter_(-1, am.unsqueeze(-1), (b["d:pool1"][:NS].float() * (mx > 0)).unsqueeze(-1))
    route = route.reshape(NS, 64, 64, 32, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(NS, 128, 128, 32)
    ref = skip_g * (y1b > 0) + route
    err = _rel(b["d:conv1b"][:NS].float(), ref)
    assert err < 2e-2, ("conv9a skip", err)
