"""Inference on an exported model (the reference's ``tf.saved_model.loader``
flow, `sanity_check_trained_model.py:38-44`).

:func:`load_saved_model` reads ``saved_model/saved_model.pb`` -- the ``serve`` tag, the
``intel_unet_brats_model`` signature's input / output tensors (``Placeholder:0`` ->
``Mask/Sigmoid:0``) and the UNet architecture recovered from the GraphDef
(:func:`utils.tf_graph.spec_from_graph`: VariableV2 shapes, pool / upsample / norm
nodes) -- and the weights from ``saved_model/variables/variables.{index,data-*}`` (TF
bundle), both written by :func:`utils.checkpoint.export_model`; the JSON side-car is
only a fallback for directories without a ``saved_model.pb``.  It returns a
:class:`Predictor` whose ``predict(x)`` maps NHWC(/NDHWC) float images to sigmoid
probabilities.

On a GPU the native HIP executor's inference plan runs (forward only, dropout
off, fused head+sigmoid) at a fixed micro-batch; a short last batch is padded.
Elsewhere, or for configs the native executor does not cover, the ATen
reference forward runs.
"""

import json
import os
from typing import Optional

import numpy as np
import torch

from .models.spec import UNetSpec
from .runtime.params import FlatParams
from .utils import tf_bundle
from .utils.checkpoint import tensors_to_flat


class _Cfg:
    """Minimal config for the backends (inference needs no optimiser flags)."""

    def __init__(self, img_size, dtype, eval_dropout=False):
        self.img_size = img_size
        self.dtype = dtype
        self.loss = "dice"
        self.bce_weight = 1.0
        self.eval_dropout = eval_dropout
        self.backend = "auto"


class Predictor:
    def __init__(self, spec: UNetSpec, flat: FlatParams, img_size: int, device, batch: int,
                 dtype: str = "bf16", backend: str = "auto", state=None):
        from .runtime.backends import NativeBackend, TorchBackend, resolve_backend
        self.spec, self.flat, self.batch, self.img_size = spec, flat, batch, img_size
        self.device = torch.device(device)
        cfg = _Cfg(img_size, dtype if self.device.type == "cuda" else "fp32")
        if resolve_backend(backend, spec, cfg, self.device) == "native":
            from . import native
            native.require()
            self.backend = NativeBackend(spec, flat, cfg, self.device, batch)
            self.backend.engine.repack()
        else:
            self.backend = TorchBackend(spec, flat, cfg, self.device, batch)
        # BatchNorm moving statistics (both backends keep them under the same names;
        # the native inference plan normalises with them)
        for k, v in (state or {}).items():
            if k in self.backend.state:
                self.backend.state[k].copy_(torch.as_tensor(np.asarray(v, np.float32)))
        self.name = self.backend.name

    @torch.no_grad()
    def predict(self, x) -> np.ndarray:
        """Probabilities for a batch of any length (native: chunks of ``batch``)."""
        x = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32))
        n = x.shape[0]
        if self.backend.name != "native":
            return self.backend.predict(x.to(self.device)).float().cpu().numpy()
        outs = []
        for s in range(0, n, self.batch):
            xb = x[s:s + self.batch]
            m = xb.shape[0]
            if m < self.batch:
                xb = torch.cat([xb, xb.new_zeros((self.batch - m,) + tuple(xb.shape[1:]))])
            p = self.backend.predict(xb.to(self.device))
            outs.append(p[:m].float().cpu())
        return torch.cat(outs).numpy()


SIGNATURE = "intel_unet_brats_model"


def _spec_from_pb(path: str):
    from .utils import tf_graph
    sm = tf_graph.read_saved_model(path)
    if "serve" not in sm["tags"]:
        raise ValueError("%s has no 'serve' meta graph" % path)
    if SIGNATURE not in sm["signatures"]:
        raise ValueError("%s has no %s signature" % (path, SIGNATURE))
    sig = sm["signatures"][SIGNATURE]
    if sig["inputs"]["image"]["name"] != "Placeholder:0" or sig["outputs"]["prediction"]["name"] != "Mask/Sigmoid:0":
        raise ValueError("unexpected signature tensors %s" % sig)
    return tf_graph.spec_from_graph(sm, SIGNATURE)


def _spec_from_json(path: str):
    with open(path) as f:
        meta = json.load(f)
    if "serve" not in meta.get("tags", []):
        raise ValueError("export %s has no 'serve' tag" % path)
    m = meta["model"]
    spec = UNetSpec(in_channels=m["in_channels"], n_cl_out=m["n_cl_out"], base=m["base"], depth=m["depth"],
                    use_upsampling=m["use_upsampling"], dims=m["dims"], dropout=m["dropout"],
                    norm=m.get("norm", "none"), groups=m.get("groups", 8))
    sig = next(iter(meta["signature_def"].values()))
    return spec, meta.get("img_size") or sig["inputs"]["image"]["shape"][1]


def load_saved_model(export_dir: str, device=None, batch: int = 128, dtype: str = "bf16",
                     backend: str = "auto") -> Predictor:
    pb = os.path.join(export_dir, "saved_model.pb")
    if os.path.exists(pb):
        spec, img_size = _spec_from_pb(pb)
    else:
        spec, img_size = _spec_from_json(os.path.join(export_dir, "saved_model.json"))
    if device is None:
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
    flat = FlatParams(spec, device=device)
    tensors = tf_bundle.read_bundle(os.path.join(export_dir, "variables", "variables"))
    tensors_to_flat(flat, tensors, strict=True)
    state = {k: v for k, v in tensors.items() if k.endswith("moving_mean") or k.endswith("moving_variance")}
    return Predictor(spec, flat, int(img_size), device, batch, dtype=dtype, backend=backend, state=state)
