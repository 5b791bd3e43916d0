"""Loss scaling for fp16 training (``--dtype fp16``).

fp16 keeps 10 mantissa bits but only 5 exponent bits: the per-pixel loss gradient
of a batch-global Dice loss is ~1 / (batch * H * W) (2.4e-7 at 256 x 128 x 128),
below fp16's normal range.  The backward therefore starts from ``loss * scale``
(the native head backward reads the scale from device memory,
``NativeUNet.set_loss_scale``), every gradient carries the factor, and the
optimizer multiplies it back out (``TFAdam.step(grad_scale=1/scale)``, fused into
the Adam kernel).

Dynamic mode (``--loss_scale 0``, default): start at 2^16; a step whose reduced
gradients are not all finite is skipped and the scale halved; after
``growth_interval`` consecutive good steps the scale doubles.  The finiteness test
runs on the allreduced gradients, so every rank takes the same decision.  Static
mode (``--loss_scale S``) never changes S but still skips non-finite steps.

The reference trains in fp32 (TF 1.4, `test_dist.py:246`) and has no equivalent;
bf16 / fp32 runs use scale 1 and no check.
"""

import torch


class LossScaler:
    def __init__(self, dtype: str, loss_scale: float = 0.0, init_scale: float = 2.0 ** 16,
                 growth_interval: int = 2000, min_scale: float = 1.0, max_scale: float = 2.0 ** 24):
        self.enabled = dtype == "fp16"
        self.dynamic = self.enabled and not loss_scale > 0
        self.scale = (float(loss_scale) if loss_scale > 0 else init_scale) if self.enabled else 1.0
        self.growth_interval = growth_interval
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.good_steps = 0
        self.skipped = 0

    def update(self, grad: torch.Tensor) -> bool:
        """Return True if the step should be applied; adjust the scale."""
        if not self.enabled:
            return True
        finite = bool(torch.isfinite(grad).all().item())
        if not finite:
            self.skipped += 1
            self.good_steps = 0
            if self.dynamic:
                self.scale = max(self.min_scale, self.scale * 0.5)
            return False
        self.good_steps += 1
        if self.dynamic and self.good_steps >= self.growth_interval:
            self.scale = min(self.max_scale, self.scale * 2.0)
            self.good_steps = 0
        return True

    def state_dict(self) -> dict:
        return {"scale": self.scale, "good_steps": self.good_steps, "skipped": self.skipped}
