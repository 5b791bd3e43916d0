"""TF V2 tensor-bundle checkpoints, TensorBoard event files, CRC32C (CPU)."""
import os
import struct

import numpy as np
import pytest
import torch

from unet_distributed_amd.utils import tf_bundle, events
from unet_distributed_amd.utils.checkpoint import CheckpointManager, flat_to_tensors, tensors_to_flat, export_model
from unet_distributed_amd.models.spec import UNetSpec, spec_from_config
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


def _graph_nodes(graph_def: bytes):
    """name -> (op, inputs, attr keys) from a GraphDef (wire-format reader)."""
    out = {}
    for nd in tf_bundle._parse(graph_def).get(1, []):
        f = tf_bundle._parse(nd)
        attrs = [tf_bundle._parse(a)[1][0].decode() for a in f.get(5, [])]
        out[f[1][0].decode()] = (f[2][0].decode(), [i.decode() for i in f.get(3, [])], attrs)
    return out


def _map(entries):
    return {tf_bundle._parse(e)[1][0].decode(): tf_bundle._parse(e).get(2, [b""])[0] for e in entries}


@pytest.mark.parametrize("kw", [dict(), dict(norm="batch"), dict(use_upsampling=True, in_channels=1),
                                dict(dims=3, in_channels=4), dict(dims=3, in_channels=4, use_upsampling=True),
                                dict(norm="group", groups=4)])
def test_saved_model_names_resolve_and_spec_roundtrips(tmp_path, kw):
    """Every name a TF loader looks up resolves to a node of the GraphDef: node inputs,
    the VariableDefs of both variable collections (variable / initializer / snapshot),
    the SaverDef's tensors and op, the SignatureDef's tensors -- in saved_model.pb and in
    a checkpoint's .meta (Adam slots, beta powers, global_step included).  The
    architecture recovered from the graph alone equals the exported spec."""
    from unet_distributed_amd.utils import tf_graph
    cfg = Config(checkpoint_dir=str(tmp_path), img_size=32 if kw.get("dims") == 3 else 64, save_model_secs=0, **kw)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    d = export_model(cfg, spec, flat)
    prefix = CheckpointManager(cfg, flat, True).save()
    for path in (os.path.join(d, "saved_model.pb"), prefix + ".meta"):
        raw = open(path, "rb").read()
        mg = tf_bundle._parse(tf_bundle._parse(raw)[2][0]) if path.endswith(".pb") else tf_bundle._parse(raw)
        nodes = tf_graph.graph_nodes(mg[2][0])

        def resolves(tensor):
            return tensor.lstrip("^").split(":")[0] in nodes

        for n, v in nodes.items():
            assert all(resolves(i) for i in v["inputs"]), (n, v["inputs"])
        for e in mg.get(4, []):
            kv = tf_bundle._parse(e)
            for vd in tf_bundle._parse(tf_bundle._parse(kv[2][0])[2][0]).get(1, []):
                f = tf_bundle._parse(vd)
                for k in (1, 2, 3):
                    assert resolves(f[k][0].decode()), (kv[1][0], k, f[k][0])
                assert nodes[f[2][0].decode()]["op"] == "Assign"
                assert nodes[f[3][0].decode().split(":")[0]]["op"] == "Identity"
        sv = tf_bundle._parse(mg[3][0])
        for k in (1, 2, 3):
            assert resolves(sv[k][0].decode()), (k, sv[k][0])
        for e in mg.get(5, []):
            sd = tf_bundle._parse(tf_bundle._parse(e)[2][0])
            for f in (1, 2):
                for te in sd.get(f, []):
                    info = tf_bundle._parse(tf_bundle._parse(te)[2][0])      # TensorInfo
                    assert resolves(info[1][0].decode()), info[1][0]
    sm = tf_graph.read_saved_model(os.path.join(d, "saved_model.pb"))
    spec2, img = tf_graph.spec_from_graph(sm)
    assert img == cfg.img_size
    for k in ("in_channels", "n_cl_out", "base", "depth", "use_upsampling", "dims", "norm", "groups"):
        assert getattr(spec2, k) == getattr(spec, k), k


@pytest.mark.parametrize("kw", [dict(), dict(norm="batch"), dict(use_upsampling=True, in_channels=1),
                                dict(dims=3, in_channels=4)])
def test_saved_model_pb_structure(tmp_path, kw):
    """export_model writes saved_model.pb: SavedModel {schema 1, MetaGraphDef tagged
    serve, signature intel_unet_brats_model image -> prediction (Placeholder:0 ->
    Mask/Sigmoid:0), a GraphDef connecting them, a V2 SaverDef}.  Parsed with the
    wire-format reader; TF-loader parity is unpinned (TF not installed)."""
    cfg = Config(checkpoint_dir=str(tmp_path), img_size=32 if kw.get("dims") == 3 else 64, **kw)
    spec = spec_from_config(cfg)
    d = export_model(cfg, spec, FlatParams(spec))
    sm = tf_bundle._parse(open(os.path.join(d, "saved_model.pb"), "rb").read())
    assert sm[1] == [1] and len(sm[2]) == 1
    mg = tf_bundle._parse(sm[2][0])
    info = tf_bundle._parse(mg[1][0])
    assert [t.decode() for t in info[4]] == ["serve"]
    sigs = _map(mg[5])
    sig = tf_bundle._parse(sigs["intel_unet_brats_model"])
    ins, outs = _map(sig[1]), _map(sig[2])
    assert tf_bundle._parse(ins["image"])[1][0] == b"Placeholder:0"
    assert tf_bundle._parse(outs["prediction"])[1][0] == b"Mask/Sigmoid:0"
    assert sig[3][0] == b"tensorflow/serving/predict"
    nodes = _graph_nodes(mg[2][0])
    assert nodes["Placeholder"][0] == "Placeholder" and nodes["Mask/Sigmoid"][0] == "Sigmoid"
    # every trainable variable is a VariableV2 restored by the saver
    for name, shape in spec.variables():
        assert nodes[name][0] == "VariableV2", name
    saver = tf_bundle._parse(mg[3][0])
    assert saver[3][0] == b"save/restore_all" and saver[7] == [2]
    assert nodes["save/restore_all"][0] == "NoOp"
    # the graph is connected: walk back from the output to the placeholder
    seen, stack = set(), ["Mask/Sigmoid"]
    while stack:
        n = stack.pop()
        if n in seen:
            continue
        seen.add(n)
        stack.extend(i.lstrip("^").split(":")[0] for i in nodes[n][1])
    assert "Placeholder" in seen and "conv1a/kernel" in seen
    if kw.get("norm") == "batch":
        assert nodes["conv1a/norm/FusedBatchNorm"][0] == "FusedBatchNorm"


def test_checkpoint_writes_saver_meta(tmp_path):
    cfg = Config(checkpoint_dir=str(tmp_path), img_size=64, save_model_secs=0)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    mgr = CheckpointManager(cfg, flat, True)
    prefix = mgr.save()
    meta = tf_bundle._parse(open(prefix + ".meta", "rb").read())
    nodes = _graph_nodes(meta[2][0])
    bundle = tf_bundle.read_bundle(prefix)
    for name in bundle:                       # weights, Adam slots, beta powers, global_step
        assert name in nodes and nodes[name][0] == "VariableV2", name
    restore = nodes["save/RestoreV2/tensor_names"]
    assert restore[0] == "Const"
    colls = _map(meta[4])
    assert "trainable_variables" in colls and "variables" in colls
    lg = mgr.save_last_good()
    assert os.path.exists(lg + ".meta")


def test_metric_logger_writes_histograms_and_images(tmp_path):
    from unet_distributed_amd.utils.metrics import MetricLogger
    cfg = Config(checkpoint_dir=str(tmp_path), log_jsonl="")
    log = MetricLogger(cfg, True, str(tmp_path / "logs"))
    m = dict(loss=0.5, dice=0.6, sensitivity=0.7, specificity=0.8, percent_complete=10.0, images_per_sec=1.0,
             lr=1e-3)
    imgs = {k: np.random.rand(3, 16, 16).astype(np.float32) for k in ("predictions", "ground_truth", "images")}
    log.train(1, m, 10, images=imgs)
    log.close()
    recs = events.read_events(log.events.path)
    tags = set(t for _, v in recs for t in v)
    for t in ("loss", "loss_1", "dice_1", "sensitivity_1", "specificity_1", "predictions/image/0",
              "ground_truth/image/2", "images/image/1"):
        assert t in tags, (t, tags)
