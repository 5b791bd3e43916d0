"""Flat parameter / gradient / optimizer-state storage.

All trainable variables live in ONE contiguous fp32 buffer laid out in
backward-ready order (Mask first ... conv1a last; ``UNetSpec.grad_ready_order``)
so that

* gradient allreduce buckets are contiguous slices of the flat gradient
  buffer (no pack/unpack kernels; SURVEY.md §2.6 bucket plan);
* the fused TF-Adam kernel is a single launch over the whole buffer
  (SURVEY.md §2.4 "ApplyAdam (x46 vars)");
* checkpoints address variables by their TF names as views of the buffer.

The reference keeps the same state as separate TF variables on the parameter
server (`test_dist.py:136-146,185,246`): weights, Adam slots ``<var>/Adam`` and
``<var>/Adam_1``, ``beta1_power``, ``beta2_power`` and ``global_step``.
"""

import math
from typing import Dict, List, Tuple

import torch

from ..models.spec import UNetSpec


class FlatParams:
    def __init__(self, spec: UNetSpec, device="cpu", align: int = 64):
        self.spec = spec
        self.device = torch.device(device)
        self.entries: List[Tuple[str, Tuple[int, ...], int, int]] = []
        off = 0
        for name, shape in spec.grad_ready_order():
            n = math.prod(shape)
            self.entries.append((name, tuple(shape), off, n))
            off += n
            off = (off + align - 1) // align * align   # keep every view 256B aligned
        self.numel = off
        self.index = {e[0]: e for e in self.entries}
        self.master = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.m = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.v = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.global_step = 0
        self.beta1_power = 0.9
        self.beta2_power = 0.999

    # ------------------------------------------------------------------
    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        _, shape, off, n = self.index[name]
        return buf[off:off + n].view(shape)

    def params(self) -> Dict[str, torch.Tensor]:
        return {e[0]: self.view(self.master, e[0]) for e in self.entries}

    def grads(self) -> Dict[str, torch.Tensor]:
        return {e[0]: self.view(self.grad, e[0]) for e in self.entries}

    def load_dict(self, d: Dict[str, torch.Tensor]) -> None:
        for name, shape, off, n in self.entries:
            src = d[name]
            if tuple(src.shape) != shape:
                raise ValueError("shape mismatch for %s: %s vs %s"
                                 % (name, tuple(src.shape), shape))
            self.master[off:off + n].copy_(src.reshape(-1).to(self.master))

    def layer_range(self, layer_name: str) -> Tuple[int, int]:
        """[start, end) of a layer's variables in the flat buffer."""
        offs = [(off, off + n) for name, _, off, n in self.entries
                if name.split("/")[0] == layer_name]
        return min(o[0] for o in offs), max(o[1] for o in offs)

    def to(self, device):
        device = torch.device(device)
        for k in ("master", "grad", "m", "v"):
            setattr(self, k, getattr(self, k).to(device))
        self.device = device
        return self
