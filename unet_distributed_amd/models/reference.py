"""PyTorch (ATen) reference implementation of the UNet forward pass.

This is the CPU path (the gloo plumbing config of BASELINE.json) and the
numerical oracle the native HIP executor is tested against.  It consumes the
same TF-layout parameter dict as the native engine and checkpoint code:
conv kernels HWIO, transposed-conv kernels ``(kh, kw, Cout, Cin)``
(`model.py:47-120`).  Activations are channels-last (NHWC / NDHWC), as in the
reference (`model.py:25-34`).

Initialisation reproduces Keras' defaults used by the reference:
``he_uniform`` for the 3x3 convs (`model.py:47-49`), ``glorot_uniform`` for
Conv2DTranspose and the 1x1 Mask conv (`model.py:79,119`), zero biases.
"""

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .spec import UNetSpec


def init_params(spec: UNetSpec, seed: int = 0, dtype=torch.float32,
                device="cpu") -> Dict[str, torch.Tensor]:
    g = torch.Generator(device="cpu").manual_seed(seed)
    params = {}
    for name, shape in spec.variables():
        layer = spec.by_name[name.split("/")[0]]
        if name.endswith("/kernel"):
            rf = math.prod(shape[:-2])
            fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
            if layer.kind == "conv":
                limit = math.sqrt(6.0 / fan_in)                 # he_uniform
            else:
                limit = math.sqrt(6.0 / (fan_in + fan_out))     # glorot_uniform
            t = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * limit
        elif name.endswith("/gamma"):
            t = torch.ones(shape, dtype=torch.float64)
        else:
            t = torch.zeros(shape, dtype=torch.float64)
        params[name] = t.to(dtype=dtype, device=device)
    return params


# ----------------------------------------------------------------------------
# layout helpers: TF kernels -> torch weight layouts
def conv_weight(k: torch.Tensor) -> torch.Tensor:
    """HWIO / DHWIO -> OIHW / OIDHW."""
    nd = k.dim() - 2
    return k.permute(nd + 1, nd, *range(nd))


def tconv_weight(k: torch.Tensor) -> torch.Tensor:
    """(kh, kw, Cout, Cin) -> torch conv_transpose weight (Cin, Cout, kh, kw)."""
    nd = k.dim() - 2
    return k.permute(nd + 1, nd, *range(nd))


def to_cf(x: torch.Tensor) -> torch.Tensor:
    """channels-last -> channels-first view."""
    nd = x.dim() - 2
    return x.permute(0, nd + 1, *range(1, nd + 1))


def to_cl(x: torch.Tensor) -> torch.Tensor:
    nd = x.dim() - 2
    return x.permute(0, *range(2, nd + 2), 1)


def dropout_keep_mask(seed: int, salt: int, shape, rate: float, device) -> torch.Tensor:
    """Counter-based keep mask shared with the HIP kernels (see csrc common.h
    ``drop_hash``): element i of a tensor is kept iff
    hash(seed, salt, i) >= rate * 2^32.  Used so the reference path and the
    native path draw identical dropout masks."""
    n = math.prod(shape)
    idx = torch.arange(n, dtype=torch.int64, device=device)
    h = _hash_u32(idx, seed, salt)
    thr = int(rate * 4294967296.0)
    return (h >= thr).reshape(shape)


def _hash_u32(idx: torch.Tensor, seed: int, salt: int) -> torch.Tensor:
    M = 0xFFFFFFFF
    x = (idx & M) ^ ((seed * 0x9E3779B9 + salt * 0x85EBCA6B) & M)
    x = x ^ ((idx >> 32) * 0xC2B2AE35 & M)
    # murmur3 fmix32
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & M
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & M
    x = x ^ (x >> 16)
    return x


def _norm(x_cf, p, name, spec: UNetSpec, train: bool, state):
    if spec.norm == "none":
        return x_cf
    gamma, beta = p[name + "/norm/gamma"], p[name + "/norm/beta"]
    if spec.norm == "group":
        return F.group_norm(x_cf, spec.groups, gamma, beta, eps=1e-3)
    rm = state.get(name + "/norm/moving_mean") if state is not None else None
    rv = state.get(name + "/norm/moving_variance") if state is not None else None
    return F.batch_norm(x_cf, rm, rv, gamma, beta, training=train or rm is None,
                        momentum=0.01, eps=1e-3)


def forward(spec: UNetSpec, p: Dict[str, torch.Tensor], x: torch.Tensor,
            train: bool = True, dropout: bool = True, seed: int = 0,
            state: Optional[dict] = None, return_logits: bool = False):
    """UNet forward.  x: channels-last [B, (D,) H, W, Cin] -> probabilities
    channels-last [B, (D,) H, W, n_cl_out] (sigmoid output, `model.py:119-120`)."""
    nd = spec.dims
    conv = F.conv2d if nd == 2 else F.conv3d
    tconv = F.conv_transpose2d if nd == 2 else F.conv_transpose3d
    pool = F.max_pool2d if nd == 2 else F.max_pool3d
    h = to_cf(x)
    acts = {}
    for salt, l in enumerate(spec.layers):     # dropout salt = layer index (same as the HIP path)
        if l.kind == "conv":
            inp = h
            if l.skip_from is not None:
                inp = torch.cat([h, acts[l.skip_from]], dim=1)
            w = conv_weight(p[l.name + "/kernel"]).to(inp.dtype)
            h = conv(inp, w, p[l.name + "/bias"].to(inp.dtype), padding=1)
            h = _norm(h, p, l.name, spec, train, state)
            h = F.relu(h)
            if l.dropout and dropout and spec.dropout > 0:
                keep = dropout_keep_mask(seed, salt, to_cl(h).shape, spec.dropout, h.device)
                h = h * to_cf(keep.to(h.dtype)) * (1.0 / (1.0 - spec.dropout))
            acts[l.name] = h
        elif l.kind == "pool":
            h = pool(h, 2)
        elif l.kind == "tconv":
            w = tconv_weight(p[l.name + "/kernel"]).to(h.dtype)
            h = tconv(h, w, p[l.name + "/bias"].to(h.dtype), stride=2)
        elif l.kind == "up":
            h = F.interpolate(h, scale_factor=2, mode="nearest")
        elif l.kind == "mask":
            w = conv_weight(p[l.name + "/kernel"]).to(h.dtype)
            h = conv(h, w, p[l.name + "/bias"].to(h.dtype))
            if not return_logits:
                h = torch.sigmoid(h)
    return to_cl(h)
