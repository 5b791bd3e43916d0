"""Checkpoint / resume / export with the reference's layout and variable names.

Layout:

* periodic saves every ``save_model_secs`` (default 60, `test_dist.py:354`) to
  ``CHECKPOINT_DIRECTORY/unet,lr=<lr>,<conv2DTranspose|upsample2D>,intra=<n>,inter=<m>/model.ckpt-<global_step>``
  (`test_dist.py:337-345`), with the ``checkpoint`` state file TF's Saver keeps
  (last 5 retained, Saver's default max_to_keep);
* ``CHECKPOINT_DIRECTORY/last_good_model.cpkt`` after every epoch's evaluation
  and at the end (`test_dist.py:446,490`; the ``.cpkt`` misspelling is kept, Q16);
* variables: ``<layer>/kernel`` (HWIO; transposed convs (kh,kw,Cout,Cin)),
  ``<layer>/bias``, Adam slots ``<var>/Adam`` and ``<var>/Adam_1``,
  ``beta1_power``, ``beta2_power`` and ``global_step`` (int64) -- everything
  the Supervisor restores (`test_dist.py:361-362`);
* every bundle gets the Saver's ``<prefix>.meta`` MetaGraphDef (graph + SaverDef +
  variable collections, hand-encoded: utils/tf_graph.py);
* export (C19, `test_dist.py:511-532`): ``CHECKPOINT_DIRECTORY/saved_model/``
  with ``saved_model.pb`` (SavedModel protobuf: tag ``serve``, signature
  ``intel_unet_brats_model`` {image: Placeholder:0 -> prediction: Mask/Sigmoid:0}),
  ``variables/variables.{index,data-00000-of-00001}`` (TF bundle) and a
  ``saved_model.json`` side-car that ``inference.py`` / ``sanity_check.py`` read.
  Format parity with TensorFlow is unpinned (TF is not installed): the files are
  verified structurally against the proto field layout, not by a TF loader.

Only rank 0 writes; writes are atomic (tmp + rename).  Restores happen on rank 0
and are broadcast to every rank (replaces ``prepare_or_wait_for_session``).
"""

import json
import os
import time
from typing import Optional

import numpy as np
import torch

from . import tf_bundle, tf_graph


def logdir_name(cfg) -> str:
    return os.path.join(cfg.checkpoint_dir, "unet,lr={},{},intra={},inter={}".format(
        cfg.learning_rate, cfg.method_up, cfg.num_threads, cfg.num_inter_threads))


def flat_to_tensors(flat, include_optimizer=True, extra_state=None):
    out = {}
    for name, shape, off, n in flat.entries:
        out[name] = flat.master[off:off + n].detach().cpu().numpy().reshape(shape).astype(np.float32)
        if include_optimizer:
            out[name + "/Adam"] = flat.m[off:off + n].detach().cpu().numpy().reshape(shape).astype(np.float32)
            out[name + "/Adam_1"] = flat.v[off:off + n].detach().cpu().numpy().reshape(shape).astype(np.float32)
    if include_optimizer:
        out["beta1_power"] = np.array(flat.beta1_power, dtype=np.float32)
        out["beta2_power"] = np.array(flat.beta2_power, dtype=np.float32)
        out["global_step"] = np.array(flat.global_step, dtype=np.int64)
    for k, v in (extra_state or {}).items():
        out[k] = v.detach().cpu().numpy().astype(np.float32)
    return out


def tensors_to_flat(flat, tensors, strict=True, extra_state=None):
    dev = flat.master.device
    for name, shape, off, n in flat.entries:
        if name not in tensors:
            if strict:
                raise KeyError("checkpoint is missing variable %s" % name)
            continue
        a = np.asarray(tensors[name], dtype=np.float32)
        if tuple(a.shape) != tuple(shape):
            raise ValueError("shape mismatch for %s: %s vs %s" % (name, a.shape, shape))
        flat.master[off:off + n].copy_(torch.from_numpy(a.reshape(-1)).to(dev))
        if name + "/Adam" in tensors:
            flat.m[off:off + n].copy_(torch.from_numpy(np.asarray(tensors[name + "/Adam"], np.float32).reshape(-1)).to(dev))
            flat.v[off:off + n].copy_(torch.from_numpy(np.asarray(tensors[name + "/Adam_1"], np.float32).reshape(-1)).to(dev))
    if "global_step" in tensors:
        flat.global_step = int(np.asarray(tensors["global_step"]))
        flat.beta1_power = float(np.asarray(tensors["beta1_power"]))
        flat.beta2_power = float(np.asarray(tensors["beta2_power"]))
    for k, t in (extra_state or {}).items():
        if k in tensors:
            t.copy_(torch.from_numpy(np.asarray(tensors[k], np.float32)).to(t.device))


def _var_shapes(tensors) -> list:
    return [(k, tuple(np.asarray(v).shape)) for k, v in tensors.items()]


def write_with_meta(prefix: str, tensors, spec, img_size: int) -> None:
    """TF V2 bundle + the Saver's .meta MetaGraphDef over the same variables."""
    tf_bundle.write_bundle(prefix, tensors)
    if spec is not None:
        tf_graph.write_meta(prefix, spec, img_size, _var_shapes(tensors))


class CheckpointManager:
    def __init__(self, cfg, flat, is_chief: bool, extra_state=None, max_to_keep: int = 5):
        self.cfg = cfg
        self.flat = flat
        self.is_chief = is_chief
        self.logdir = logdir_name(cfg)
        self.max_to_keep = max_to_keep
        self.last_save = time.time()
        self.pre_save = None
        self.extra_state = extra_state or {}
        if is_chief and not cfg.no_checkpoint:
            os.makedirs(self.logdir, exist_ok=True)

    # -------------------------------------------------------------- periodic
    def maybe_save(self, force=False) -> Optional[str]:
        if self.cfg.no_checkpoint or not self.is_chief:
            return None
        if not force and time.time() - self.last_save < self.cfg.save_model_secs:
            return None
        return self.save()

    def save(self) -> Optional[str]:
        if self.cfg.no_checkpoint or not self.is_chief:
            return None
        if self.pre_save is not None:
            self.pre_save()                 # e.g. async PS: pull server state into flat
        step = self.flat.global_step
        prefix = os.path.join(self.logdir, "model.ckpt-%d" % step)
        write_with_meta(prefix, flat_to_tensors(self.flat, extra_state=self.extra_state),
                        getattr(self.flat, "spec", None), self.cfg.img_size)
        _, paths = tf_bundle.read_checkpoint_state(self.logdir)
        name = os.path.basename(prefix)
        paths = [p for p in paths if p != name] + [name]
        for old in paths[:-self.max_to_keep]:
            for suf in (".index", ".data-00000-of-00001", ".meta"):
                try:
                    os.remove(os.path.join(self.logdir, old + suf))
                except FileNotFoundError:
                    pass
        paths = paths[-self.max_to_keep:]
        tf_bundle.write_checkpoint_state(self.logdir, name, paths)
        self.last_save = time.time()
        return prefix

    def save_last_good(self) -> Optional[str]:
        if self.cfg.no_checkpoint or not self.is_chief:
            return None
        if self.pre_save is not None:
            self.pre_save()                 # async PS: the bundle must hold the server's state
        prefix = os.path.join(self.cfg.checkpoint_dir, "last_good_model.cpkt")
        write_with_meta(prefix, flat_to_tensors(self.flat, extra_state=self.extra_state),
                        getattr(self.flat, "spec", None), self.cfg.img_size)
        tf_bundle.write_checkpoint_state(self.cfg.checkpoint_dir, "last_good_model.cpkt",
                                         ["last_good_model.cpkt"])
        return prefix

    # -------------------------------------------------------------- restore
    def latest(self) -> Optional[str]:
        latest, _ = tf_bundle.read_checkpoint_state(self.logdir)
        if latest is None:
            return None
        p = latest if os.path.isabs(latest) else os.path.join(self.logdir, latest)
        return p if os.path.exists(p + ".index") else None

    def restore_latest(self) -> bool:
        p = self.latest()
        if p is None:
            return False
        tensors_to_flat(self.flat, tf_bundle.read_bundle(p), extra_state=self.extra_state)
        return True


def export_model(cfg, spec, flat, directory: Optional[str] = None, extra_state=None) -> str:
    """SavedModel-style export (C19): weights bundle + graph/signature description.
    ``extra_state``: non-trainable inference state (BatchNorm moving statistics)."""
    d = directory or os.path.join(cfg.checkpoint_dir, "saved_model")
    os.makedirs(os.path.join(d, "variables"), exist_ok=True)
    tf_bundle.write_bundle(os.path.join(d, "variables", "variables"),
                           flat_to_tensors(flat, include_optimizer=False, extra_state=extra_state))
    meta = {
        "tags": ["serve"],
        "signature_def": {"intel_unet_brats_model": {
            "inputs": {"image": {"name": "Placeholder:0", "dtype": "float32",
                                 "shape": [-1] + [cfg.img_size] * spec.dims + [spec.in_channels]}},
            "outputs": {"prediction": {"name": "Mask/Sigmoid:0", "dtype": "float32",
                                       "shape": [-1] + [cfg.img_size] * spec.dims + [spec.n_cl_out]}},
            "method_name": "tensorflow/serving/predict"}},
        "img_size": cfg.img_size,
        "model": {"in_channels": spec.in_channels, "n_cl_out": spec.n_cl_out, "base": spec.base,
                  "depth": spec.depth, "use_upsampling": spec.use_upsampling, "dims": spec.dims,
                  "dropout": spec.dropout, "norm": spec.norm, "groups": spec.groups},
    }
    with open(os.path.join(d, "saved_model.json"), "w") as f:
        json.dump(meta, f, indent=2)
    tf_graph.write_saved_model(d, spec, cfg.img_size)
    return d
