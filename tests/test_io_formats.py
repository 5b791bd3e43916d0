"""TF V2 tensor-bundle checkpoints, TensorBoard event files, CRC32C (CPU)."""
import os
import struct

import numpy as np
import pytest
import torch

from unet_distributed_amd.utils import tf_bundle, events
from unet_distributed_amd.utils.checkpoint import CheckpointManager, flat_to_tensors, tensors_to_flat, export_model
from unet_distributed_amd.models.spec import UNetSpec
from unet_distributed_amd.models import reference
from unet_distributed_amd.runtime.params import FlatParams
from unet_distributed_amd.config import Config


def test_crc32c_known_vectors():
    assert tf_bundle.crc32c(b"123456789") == 0xE3069283
    assert tf_bundle._py_crc32c(b"123456789") == 0xE3069283
    assert tf_bundle.crc32c(b"") == 0
    m = tf_bundle.mask_crc(0xE3069283)
    assert tf_bundle.unmask_crc(m) == 0xE3069283


def test_native_crc_matches_python_on_random_bytes():
    data = np.random.default_rng(0).integers(0, 256, 10007, dtype=np.uint8).tobytes()
    assert tf_bundle.crc32c(data) == tf_bundle._py_crc32c(data)


def test_bundle_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    t = {"conv1a/kernel": rng.standard_normal((3, 3, 1, 32)).astype(np.float32),
         "conv1a/bias": np.zeros(32, np.float32),
         "global_step": np.array(17, np.int64),
         "beta1_power": np.array(0.9 ** 17, np.float32)}
    prefix = str(tmp_path / "model.ckpt-17")
    tf_bundle.write_bundle(prefix, t)
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001")
    r = tf_bundle.read_bundle(prefix)
    assert set(r) == set(t)
    for k in t:
        assert r[k].dtype == t[k].dtype and r[k].shape == t[k].shape
        assert np.array_equal(r[k], t[k])


def test_bundle_index_structure(tmp_path):
    prefix = str(tmp_path / "x")
    tf_bundle.write_bundle(prefix, {"a": np.ones(3, np.float32)})
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == tf_bundle.TABLE_MAGIC
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    assert data == np.ones(3, np.float32).tobytes()


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path / "x")
    tf_bundle.write_bundle(prefix, {"a": np.arange(16, dtype=np.float32)})
    p = prefix + ".data-00000-of-00001"
    b = bytearray(open(p, "rb").read())
    b[5] ^= 0xFF
    open(p, "wb").write(bytes(b))
    with pytest.raises(IOError):
        tf_bundle.read_bundle(prefix)


def test_checkpoint_state_file(tmp_path):
    tf_bundle.write_checkpoint_state(str(tmp_path), "model.ckpt-20", ["model.ckpt-10", "model.ckpt-20"])
    latest, paths = tf_bundle.read_checkpoint_state(str(tmp_path))
    assert latest == "model.ckpt-20" and paths == ["model.ckpt-10", "model.ckpt-20"]


def test_checkpoint_manager_save_restore(tmp_path):
    cfg = Config(checkpoint_dir=str(tmp_path), save_model_secs=0)
    spec = UNetSpec()
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=0))
    flat.m.normal_()
    flat.v.uniform_()
    flat.global_step, flat.beta1_power, flat.beta2_power = 42, 0.9 ** 43, 0.999 ** 43
    mgr = CheckpointManager(cfg, flat, is_chief=True)
    prefix = mgr.save()
    assert os.path.basename(prefix) == "model.ckpt-42"
    assert "unet,lr=0.0005,conv2DTranspose,intra=50,inter=2" in prefix
    names = set(tf_bundle.read_bundle(prefix))
    assert {"conv1a/kernel", "conv1a/kernel/Adam", "conv1a/kernel/Adam_1", "beta1_power", "beta2_power",
            "global_step", "transConv6/kernel"} <= names
    flat2 = FlatParams(spec)
    mgr2 = CheckpointManager(cfg, flat2, is_chief=True)
    assert mgr2.restore_latest()
    for name, shape, off, n in flat.entries:     # (alignment padding between variables is not saved)
        assert torch.equal(flat2.m[off:off + n], flat.m[off:off + n])
    assert torch.equal(flat2.master, flat.master)
    assert flat2.global_step == 42 and abs(flat2.beta1_power - 0.9 ** 43) < 1e-7
    lg = mgr.save_last_good()
    assert lg.endswith("last_good_model.cpkt") and os.path.exists(lg + ".index")


def test_checkpoint_keeps_last_five(tmp_path):
    cfg = Config(checkpoint_dir=str(tmp_path), save_model_secs=0)
    spec = UNetSpec(base=32)
    flat = FlatParams(spec)
    mgr = CheckpointManager(cfg, flat, is_chief=True)
    for s in range(7):
        flat.global_step = s
        mgr.save()
    latest, paths = tf_bundle.read_checkpoint_state(mgr.logdir)
    assert latest == "model.ckpt-6" and len(paths) == 5
    assert not os.path.exists(os.path.join(mgr.logdir, "model.ckpt-0.index"))


def test_export_model(tmp_path):
    cfg = Config(checkpoint_dir=str(tmp_path))
    spec = UNetSpec()
    flat = FlatParams(spec)
    d = export_model(cfg, spec, flat)
    assert os.path.exists(os.path.join(d, "variables", "variables.index"))
    import json
    meta = json.load(open(os.path.join(d, "saved_model.json")))
    assert "intel_unet_brats_model" in meta["signature_def"]


def test_event_file_roundtrip(tmp_path):
    w = events.EventWriter(str(tmp_path))
    w.scalars(3, {"loss": 0.5, "dice": 0.25})
    w.histogram(3, "loss", [0.1, 0.2, 0.3])
    w.images(3, "predictions", np.random.rand(4, 16, 16, 1), max_outputs=3)
    w.close()
    recs = events.read_events(w.path)
    assert recs[0][1] == {}      # file_version record
    scal = [r for r in recs if "loss" in r[1] and r[1]["loss"] is not None]
    assert scal and abs(scal[0][1]["loss"] - 0.5) < 1e-7 and scal[0][0] == 3


def test_png_encoder_produces_valid_signature():
    png = events.png_gray(np.arange(64, dtype=np.uint8).reshape(8, 8))
    assert png[:8] == b"\x89PNG\r\n\x1a\n" and b"IEND" in png
