"""Static description of the UNet graph (layer names, channel widths, shapes).

The layer list reproduces the reference's Keras graph (`model.py:36-130`):

* encoder levels 1..depth: ``conv{i}a`` / ``conv{i}b`` (3x3, ReLU, he_uniform),
  dropout after ``conv{depth-1}a`` and ``conv{depth}a`` (`model.py:60,66`),
  2x2 max-pool after each ``conv{i}b`` (`model.py:53-69`);
* bottleneck ``conv{depth+1}a`` / ``conv{depth+1}b`` (`model.py:71-78`);
* decoder levels depth+2..2*depth+1: ``transConv{j}`` (2x2 stride 2, linear,
  glorot_uniform; `model.py:79-113`) or nearest ``up{j}`` (upsampling
  variant), channel-concat with the encoder skip, ``conv{j}a`` / ``conv{j}b``;
* ``Mask``: 1x1 conv + sigmoid (`model.py:119-120`).

Variable names and kernel layouts are the TF ones: conv kernels are HWIO
(``(kh, kw, Cin, Cout)``, ``(kd, kh, kw, Cin, Cout)`` in 3D) and transposed
conv kernels are ``(kh, kw, Cout, Cin)`` (Keras Conv2DTranspose).  These are
what the checkpoint stores.

The same spec drives the PyTorch reference implementation, the native HIP
executor, parameter-count tests and allreduce bucket planning.
"""

import dataclasses
import math
from typing import Dict, List, Optional, Tuple


@dataclasses.dataclass
class Layer:
    name: str
    kind: str                    # conv | tconv | up | pool | mask
    cin: int
    cout: int
    level: int                   # spatial level (1 = full resolution)
    relu: bool = True
    dropout: bool = False
    skip_from: Optional[str] = None   # decoder conv{j}a: name of the skip tensor
    up_channels: int = 0              # decoder conv{j}a: channels coming from up-path
    ksize: int = 3

    def kernel_shape(self, dims: int) -> Tuple[int, ...]:
        if self.kind == "conv":
            return (self.ksize,) * dims + (self.cin, self.cout)
        if self.kind == "tconv":
            return (2,) * dims + (self.cout, self.cin)
        if self.kind == "mask":
            return (1,) * dims + (self.cin, self.cout)
        raise ValueError(self.kind)

    @property
    def has_params(self) -> bool:
        return self.kind in ("conv", "tconv", "mask")


@dataclasses.dataclass
class UNetSpec:
    in_channels: int = 1
    n_cl_out: int = 1
    base: int = 32
    depth: int = 4
    use_upsampling: bool = False
    dims: int = 2
    dropout: float = 0.2
    norm: str = "none"            # none | batch | group  [EXT]
    groups: int = 8

    def __post_init__(self):
        self.layers: List[Layer] = self._build()
        self.by_name: Dict[str, Layer] = {l.name: l for l in self.layers}

    # ------------------------------------------------------------------
    def width(self, level: int) -> int:
        return self.base * (1 << (level - 1))

    def _build(self) -> List[Layer]:
        d = self.depth
        L: List[Layer] = []
        cin = self.in_channels
        for i in range(1, d + 1):
            w = self.width(i)
            drop = self.dropout > 0 and i in (d - 1, d)
            L.append(Layer("conv%da" % i, "conv", cin, w, i, dropout=drop))
            L.append(Layer("conv%db" % i, "conv", w, w, i))
            L.append(Layer("pool%d" % i, "pool", w, w, i))
            cin = w
        bw = self.width(d + 1)
        L.append(Layer("conv%da" % (d + 1), "conv", cin, bw, d + 1))
        bout = bw // 2 if self.use_upsampling else bw
        L.append(Layer("conv%db" % (d + 1), "conv", bw, bout, d + 1))
        prev = bout
        for j in range(d + 2, 2 * d + 2):
            lvl = 2 * d + 2 - j              # 6 -> 4, ..., 9 -> 1 for depth 4
            w = self.width(lvl)
            if self.use_upsampling:
                L.append(Layer("up%d" % j, "up", prev, prev, lvl))
                upc = prev
            else:
                L.append(Layer("transConv%d" % j, "tconv", prev, w, lvl, relu=False, ksize=2))
                upc = w
            skip = "conv%db" % lvl
            L.append(Layer("conv%da" % j, "conv", upc + w, w, lvl,
                           skip_from=skip, up_channels=upc))
            last = j == 2 * d + 1
            bo = w // 2 if (self.use_upsampling and not last) else w
            L.append(Layer("conv%db" % j, "conv", w, bo, lvl))
            prev = bo
        L.append(Layer("Mask", "mask", prev, self.n_cl_out, 1, relu=False, ksize=1))
        return L

    # ------------------------------------------------------------------
    def param_layers(self) -> List[Layer]:
        return [l for l in self.layers if l.has_params]

    def variables(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """(name, shape) of every trainable variable in TF naming, forward order."""
        out = []
        for l in self.param_layers():
            out.append((l.name + "/kernel", l.kernel_shape(self.dims)))
            out.append((l.name + "/bias", (l.cout,)))
            if self.norm != "none" and l.kind == "conv":
                out.append((l.name + "/norm/gamma", (l.cout,)))
                out.append((l.name + "/norm/beta", (l.cout,)))
        return out

    def grad_ready_order(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """Variables in the order their gradients become ready in backward
        (Mask first, conv1a last).  The flat parameter / gradient buffers use
        this order so allreduce buckets are contiguous slices."""
        by_layer: Dict[str, List[Tuple[str, Tuple[int, ...]]]] = {}
        for n, s in self.variables():
            by_layer.setdefault(n.split("/")[0], []).append((n, s))
        order = []
        for l in reversed(self.param_layers()):
            order.extend(by_layer[l.name])
        return order

    def num_params(self) -> int:
        return sum(math.prod(s) for _, s in self.variables())

    def fwd_flops_per_sample(self, img: int) -> float:
        """Forward FLOPs (2*MAC) for one sample of spatial size img^dims."""
        total = 0.0
        for l in self.param_layers():
            side = img >> (l.level - 1)
            if l.kind == "tconv":
                side = side // 2          # GEMM over the low-res input pixels
            pix = side ** self.dims
            k = 1
            for s in l.kernel_shape(self.dims)[:-2]:
                k *= s
            total += 2.0 * pix * k * l.cin * l.cout
        return total


def spec_from_config(cfg) -> UNetSpec:
    return UNetSpec(in_channels=cfg.in_channels, n_cl_out=cfg.out_channels,
                    base=cfg.base_filters, depth=cfg.depth,
                    use_upsampling=cfg.use_upsampling, dims=cfg.dims,
                    dropout=cfg.dropout, norm=cfg.norm, groups=cfg.groups)
