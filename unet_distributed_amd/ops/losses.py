"""Loss and metric definitions (PyTorch reference forms).

Exact semantics of the reference (`model.py:4-21`, `model.py:133-143`):

* ``dice_coef = (2*sum(t*p) + s) / (sum(t) + sum(p) + s)`` with ``s = 1`` and
  the sums over the WHOLE batch tensor (batch, spatial and channel together);
* ``dice_coef_loss = -log(2*sum(t*p) + s) + log(sum(t) + sum(p) + s)``;
* ``sensitivity = (I + s) / (sum(t) + s)``; ``specificity = (I + s) / (sum(p) + s)``
  (the reference's "specificity" is really precision; reproduced as-is).

[EXT] ``dice_bce``: Dice loss + ``bce_weight * mean(BCE(logit, t))``, computed
from the logit for stability.  The native fused head kernel
(``csrc/kernels/head.hip``) produces the same partial sums {I, St, Sp, BCE}.
"""

import torch
import torch.nn.functional as F

SMOOTH = 1.0


def dice_sums(t: torch.Tensor, p: torch.Tensor):
    t = t.float()
    p = p.float()
    return (t * p).sum(), t.sum(), p.sum()


def dice_coef(t, p, smooth=SMOOTH):
    i, st, sp = dice_sums(t, p)
    return (2.0 * i + smooth) / (st + sp + smooth)


def dice_coef_loss(t, p, smooth=SMOOTH):
    i, st, sp = dice_sums(t, p)
    return -torch.log(2.0 * i + smooth) + torch.log(st + sp + smooth)


def sensitivity(t, p, smooth=SMOOTH):
    i, st, _ = dice_sums(t, p)
    return (i + smooth) / (st + smooth)


def specificity(t, p, smooth=SMOOTH):
    i, _, sp = dice_sums(t, p)
    return (i + smooth) / (sp + smooth)


def metrics_from_sums(i, st, sp, smooth=SMOOTH):
    """All four reference metrics from the three batch sums (floats or 0-d)."""
    dice = (2.0 * i + smooth) / (st + sp + smooth)
    return {
        "loss": -torch.log(torch.as_tensor(2.0 * i + smooth)).item()
        + torch.log(torch.as_tensor(st + sp + smooth)).item(),
        "dice": float(dice),
        "sensitivity": float((i + smooth) / (st + smooth)),
        "specificity": float((i + smooth) / (sp + smooth)),
    }


def total_loss(t, logits, kind="dice", bce_weight=1.0):
    """Training loss from logits (sigmoid applied here)."""
    p = torch.sigmoid(logits.float())
    loss = dice_coef_loss(t, p)
    if kind == "dice_bce":
        loss = loss + bce_weight * F.binary_cross_entropy_with_logits(
            logits.float(), t.float())
    return loss, p


def sanity_dice(a, b):
    """The post-hoc check's Dice (`sanity_check_trained_model.py:30-35`):
    2*(sum(a*b) + 1) / (sum(a + b) + 1) -- a different smoothing."""
    a = torch.as_tensor(a).reshape(-1).double()
    b = torch.as_tensor(b).reshape(-1).double()
    return float(2.0 * ((a * b).sum() + 1.0) / ((a + b).sum() + 1.0))
