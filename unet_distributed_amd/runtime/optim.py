"""TF-1.x-semantics Adam over the flat parameter buffer.

`test_dist.py:246` uses ``tf.train.AdamOptimizer(lr)`` with TF defaults
beta1=0.9, beta2=0.999, epsilon=1e-8, whose update is::

    lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
    m    = beta1 * m + (1 - beta1) * g
    v    = beta2 * v + (1 - beta2) * g^2
    w   -= lr_t * m / (sqrt(v) + epsilon)

Epsilon is added to the *uncorrected* sqrt(v), unlike ``torch.optim.Adam``.
``beta1_power``/``beta2_power`` are tracked like TF's slot variables (they
start at beta1/beta2 and are multiplied after every apply).

The learning-rate schedule follows `test_dist.py:228-232`: constant, or
``lr * lr_fraction ** (global_step / decay_steps)`` (continuous decay).

On the GPU the update is ONE fused HIP launch (``csrc/kernels/adam.hip``) that
also refreshes the bf16 weight copies the conv kernels consume; on CPU the
same math runs as torch vector ops.
"""

import math

import torch

BETA1 = 0.9
BETA2 = 0.999
EPSILON = 1e-8


def learning_rate(cfg, global_step: int) -> float:
    if cfg.const_learningrate:
        return float(cfg.learning_rate)
    return float(cfg.learning_rate) * (cfg.lr_fraction ** (global_step / float(cfg.decay_steps)))


def adam_reference_(w, g, m, v, lr, beta1_power, beta2_power,
                    beta1=BETA1, beta2=BETA2, eps=EPSILON):
    """In-place TF Adam on tensors (the numerical oracle)."""
    lr_t = lr * math.sqrt(1.0 - beta2_power) / (1.0 - beta1_power)
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    w.addcdiv_(m, v.sqrt().add_(eps), value=-lr_t)


class TFAdam:
    def __init__(self, flat, cfg, native=None):
        self.flat = flat
        self.cfg = cfg
        self.native = native   # runtime.native_step.NativeWeights or None

    def step(self, grad_scale: float = 1.0):
        f = self.flat
        lr = learning_rate(self.cfg, f.global_step)
        if self.native is not None:
            self.native.adam_step(lr, f.beta1_power, f.beta2_power, grad_scale)
        else:
            g = f.grad if grad_scale == 1.0 else f.grad * grad_scale
            adam_reference_(f.master, g, f.m, f.v, lr, f.beta1_power, f.beta2_power)
        f.beta1_power *= BETA1
        f.beta2_power *= BETA2
        f.global_step += 1
        return lr
