"""Model spec, loss/metric formulas and TF-Adam semantics (CPU)."""
import math

import numpy as np
import pytest
import torch

from unet_distributed_amd.models.spec import UNetSpec
from unet_distributed_amd.models import reference
from unet_distributed_amd.ops import losses
from unet_distributed_amd.runtime.optim import adam_reference_, learning_rate, TFAdam
from unet_distributed_amd.runtime.params import FlatParams
from unet_distributed_amd.config import Config


def test_param_counts_match_reference_graph():
    # 7,759,521 (Conv2DTranspose) / 5,495,521 (UpSampling2D); 4-ch input 7,760,385
    assert UNetSpec().num_params() == 7759521
    assert UNetSpec(use_upsampling=True).num_params() == 5495521
    assert UNetSpec(in_channels=4).num_params() == 7760385


def test_variable_names_and_layouts():
    v = dict(UNetSpec().variables())
    assert v["conv1a/kernel"] == (3, 3, 1, 32)
    assert v["transConv6/kernel"] == (2, 2, 256, 512)      # Keras (kh, kw, Cout, Cin)
    assert v["conv6a/kernel"] == (3, 3, 512, 256)
    assert v["Mask/kernel"] == (1, 1, 32, 1)
    assert len(v) == 46


def test_grad_ready_order_is_reverse_layer_order():
    order = [n for n, _ in UNetSpec().grad_ready_order()]
    assert order[0] == "Mask/kernel" and order[-1] == "conv1a/bias"


def test_fwd_flops():
    assert abs(UNetSpec().fwd_flops_per_sample(128) / 1e9 - 6.017) < 0.01


def test_init_bounds():
    spec = UNetSpec()
    p = reference.init_params(spec, seed=0)
    k = p["conv3a/kernel"]
    assert k.abs().max() <= math.sqrt(6.0 / (9 * 64)) + 1e-7           # he_uniform
    t = p["transConv6/kernel"]
    assert t.abs().max() <= math.sqrt(6.0 / (4 * 256 + 4 * 512)) + 1e-7  # glorot_uniform
    assert float(p["conv3a/bias"].abs().sum()) == 0.0


def test_reference_forward_shapes_and_range():
    spec = UNetSpec(in_channels=4)
    p = reference.init_params(spec, seed=0)
    x = torch.randn(2, 32, 32, 4)
    y = reference.forward(spec, p, x, train=False, dropout=False)
    assert y.shape == (2, 32, 32, 1)
    assert float(y.min()) >= 0 and float(y.max()) <= 1


def test_dice_formulas_match_numpy():
    rng = np.random.default_rng(0)
    t = (rng.random((4, 8, 8, 1)) > 0.6).astype(np.float32)
    p = rng.random((4, 8, 8, 1)).astype(np.float32)
    I, St, Sp = (t * p).sum(), t.sum(), p.sum()
    tt, pp = torch.from_numpy(t), torch.from_numpy(p)
    assert abs(float(losses.dice_coef(tt, pp)) - (2 * I + 1) / (St + Sp + 1)) < 1e-5
    assert abs(float(losses.dice_coef_loss(tt, pp)) - (-math.log(2 * I + 1) + math.log(St + Sp + 1))) < 1e-5
    assert abs(float(losses.sensitivity(tt, pp)) - (I + 1) / (St + 1)) < 1e-5
    assert abs(float(losses.specificity(tt, pp)) - (I + 1) / (Sp + 1)) < 1e-5
    assert abs(losses.sanity_dice(t, p) - 2 * ((t * p).sum() + 1) / ((t + p).sum() + 1)) < 1e-6


def test_dice_loss_gradient_formula():
    # dL/dp = -2t/(2I+1) + 1/(St+Sp+1)  (used by the fused head backward kernel)
    t = (torch.rand(64) > 0.5).float()
    p = torch.rand(64, requires_grad=True)
    L = losses.dice_coef_loss(t, p)
    (g,) = torch.autograd.grad(L, p)
    I, St, Sp = (t * p).sum(), t.sum(), p.sum()
    ref = -2 * t / (2 * I + 1) + 1 / (St + Sp + 1)
    assert torch.allclose(g, ref.detach(), atol=1e-6)


def _np_tf_adam(w, g, m, v, lr, t, b1=0.9, b2=0.999, eps=1e-8):
    lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    return w - lr_t * m / (np.sqrt(v) + eps), m, v


def test_tf_adam_matches_numpy_oracle_over_steps():
    rng = np.random.default_rng(1)
    w = rng.standard_normal(100)
    m = np.zeros(100)
    v = np.zeros(100)
    tw, tm, tv = torch.tensor(w), torch.zeros(100, dtype=torch.float64), torch.zeros(100, dtype=torch.float64)
    b1p, b2p = 0.9, 0.999
    for t in range(1, 6):
        g = rng.standard_normal(100)
        w, m, v = _np_tf_adam(w, g, m, v, 5e-4, t)
        adam_reference_(tw, torch.tensor(g), tm, tv, 5e-4, b1p, b2p)
        b1p *= 0.9
        b2p *= 0.999
    assert np.allclose(tw.numpy(), w, atol=1e-12)


def test_tf_adam_epsilon_placement_differs_from_torch():
    # eps on the UNcorrected sqrt(v): with tiny gradients the TF step is smaller than torch's
    w = torch.zeros(1, dtype=torch.float64)
    m = torch.zeros(1, dtype=torch.float64)
    v = torch.zeros(1, dtype=torch.float64)
    adam_reference_(w, torch.tensor([1e-6], dtype=torch.float64), m, v, 1.0, 0.9, 0.999)
    lr_t = math.sqrt(1 - 0.999) / (1 - 0.9)
    expect = -lr_t * (0.1 * 1e-6) / (math.sqrt(0.001 * 1e-12) + 1e-8)
    assert abs(float(w) - expect) < 1e-12


def test_lr_schedule():
    cfg = Config(const_learningrate=True, learning_rate=5e-4)
    assert learning_rate(cfg, 1000) == 5e-4
    cfg = Config(const_learningrate=False, learning_rate=1e-3, lr_fraction=0.2, decay_steps=100)
    assert abs(learning_rate(cfg, 50) - 1e-3 * 0.2 ** 0.5) < 1e-12    # continuous (staircase=False)


def test_flat_params_views_and_optimizer_state():
    spec = UNetSpec()
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=0))
    v = flat.view(flat.master, "conv5b/kernel")
    assert v.shape == (3, 3, 512, 512)
    assert (v.data_ptr() - flat.master.data_ptr()) % 256 == 0
    opt = TFAdam(flat, Config())
    flat.grad.normal_()
    opt.step()
    assert flat.global_step == 1 and abs(flat.beta1_power - 0.81) < 1e-12


def test_loss_scaler_dynamic_skip_halve_grow():
    from unet_distributed_amd.runtime.amp import LossScaler
    off = LossScaler("bf16")
    assert not off.enabled and off.scale == 1.0 and off.update(torch.tensor([float("inf")]))
    s = LossScaler("fp16", growth_interval=3)
    assert s.dynamic and s.scale == 2.0 ** 16
    assert not s.update(torch.tensor([1.0, float("nan")]))
    assert s.scale == 2.0 ** 15 and s.skipped == 1
    for _ in range(3):
        assert s.update(torch.ones(4))
    assert s.scale == 2.0 ** 16
    st = LossScaler("fp16", loss_scale=128.0)
    assert not st.dynamic and st.scale == 128.0
    assert not st.update(torch.tensor([float("inf")])) and st.scale == 128.0


def test_one_gpu_path_no_silent_aten_dispatch():
    """--backend auto on a GPU is the HIP executor or an error naming the reason, never a
    silent ATen / MIOpen run; ATen only when asked for (--backend torch)
    or off the GPU (the CPU / gloo plumbing config).  device 'cuda' is only a device
    type here: nothing touches a GPU."""
    import pytest
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.runtime.backends import resolve_backend
    ok = Config(dtype="bf16", in_channels=4)
    assert resolve_backend("auto", spec_from_config(ok), ok, "cuda") == "native"
    assert resolve_backend("auto", spec_from_config(ok), ok, "cpu") == "torch"
    assert resolve_backend("torch", spec_from_config(ok), ok, "cuda") == "torch"
    fp32 = Config(dtype="fp32", in_channels=4)          # the fp32 executor (runtime/f32_engine.py)
    assert resolve_backend("auto", spec_from_config(fp32), fp32, "cuda") == "native"
    for bad, why in ((Config(dtype="fp32", norm="batch"), "norm-free"), (Config(base_filters=48), "base filters")):
        spec = spec_from_config(bad)
        for want in ("auto", "native"):
            with pytest.raises(RuntimeError, match=why):
                resolve_backend(want, spec, bad, "cuda")
        assert resolve_backend("torch", spec, bad, "cuda") == "torch"
        assert resolve_backend("auto", spec, bad, "cpu") == "torch"
