"""Aux tools: MetaImage IO, BraTS preprocessing, export -> sanity check (CPU).

Parity is pinned against the reference's documented semantics (file:line in
the module docstrings); SimpleITK/cv2 are not installed, so the .mha inputs are
synthetic volumes written by our own writer."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from unet_distributed_amd.data import mha, preprocess  # noqa: E402


@pytest.mark.parametrize("dtype,compress", [(np.int16, False), (np.uint8, True), (np.float32, False)])
def test_mha_roundtrip(tmp_path, dtype, compress):
    a = (np.random.RandomState(0).rand(5, 7, 9) * 100).astype(dtype)
    p = str(tmp_path / "v.mha")
    mha.write_mha(p, a, spacing=[1, 1, 2], compress=compress)
    img = mha.read_mha(p)
    assert img.array.dtype == dtype and img.array.shape == (5, 7, 9)
    np.testing.assert_array_equal(img.array, a)
    assert img.GetSize() == (9, 7, 5) and img.spacing == (1.0, 1.0, 2.0)


def _make_case(root, name, depth, H, W, seed):
    rs = np.random.RandomState(seed)
    case = os.path.join(root, name)
    for k, series in enumerate(["T1", "T1c", "Flair", "T2"]):
        d = os.path.join(case, "VSD.Brain.XX.O.MR_%s.%d" % (series, 100 + k))
        os.makedirs(d)
        vol = (rs.rand(depth, H, W) * 1000 + 1000 * k).astype(np.int16)
        mha.write_mha(os.path.join(d, "VSD.Brain.XX.O.MR_%s.%d.mha" % (series, 100 + k)), vol)
    d = os.path.join(case, "VSD.Brain_3more.XX.O.OT.200")
    os.makedirs(d)
    lab = rs.randint(0, 5, size=(depth, H, W)).astype(np.uint8)
    mha.write_mha(os.path.join(d, "VSD.Brain_3more.XX.O.OT.200.mha"), lab, compress=True)
    return lab


def test_preprocess_split_crop_normalize_flip(tmp_path):
    src, out = str(tmp_path / "brats"), str(tmp_path / "out")
    labs = {}
    for i in range(6):
        labs[i] = _make_case(src, "case%02d" % i, depth=10, H=20, W=24, seed=i)
    ntr, nte = preprocess.create_datasets(src, out, img_rows=16, img_cols=16, slice_by=5, verbose=False)
    # cases 0 and 5 are test (i % 5 == 0); 2 kept slices per case (n = 5, 10)
    assert (ntr, nte) == (8, 4)
    xi = np.load(os.path.join(out, "imgs_train.npy"))
    yi = np.load(os.path.join(out, "msks_train.npy"))
    xt = np.load(os.path.join(out, "imgs_test.npy"))
    yt = np.load(os.path.join(out, "msks_test.npy"))
    assert xi.shape == (8, 16, 16, 4) and yt.shape == (4, 16, 16, 4) and xi.dtype == np.float32
    # test slice 0 = case00 slice index 4, crop rows (20-16)//2=2.., cols (24-16)//2=4..
    l0 = labs[0][4, 2:18, 4:20]
    for k in range(4):
        np.testing.assert_array_equal(yt[0, :, :, k], (l0 == k + 1).astype(np.float32))
    # training slice 1 is mirrored (cv2.flip(..., 1)); slice 0 is not
    l1 = labs[1]
    np.testing.assert_array_equal(yi[0, :, :, 1], (l1[4, 2:18, 4:20] == 2).astype(np.float32))
    np.testing.assert_array_equal(yi[1, :, :, 1], (l1[9, 2:18, 4:20] == 2).astype(np.float32)[:, ::-1])
    # per-volume z-score: a whole case volume has mean 0 / std 1 per channel (before slicing)
    img, _, complete = preprocess.case_arrays(os.path.join(src, "case01"), 16, 16)
    assert complete
    np.testing.assert_allclose(img.reshape(-1, 4).mean(0), 0, atol=1e-5)
    np.testing.assert_allclose(img.reshape(-1, 4).std(0), 1, atol=1e-4)


def test_export_then_sanity_check_matches_direct_forward(tmp_path, capsys):
    from unet_distributed_amd import sanity_check
    from unet_distributed_amd.config import Config
    from unet_distributed_amd.data.datasets import synthetic_brats
    from unet_distributed_amd.inference import load_saved_model
    from unet_distributed_amd.models import reference
    from unet_distributed_amd.models.spec import spec_from_config
    from unet_distributed_amd.ops.losses import sanity_dice
    from unet_distributed_amd.runtime.params import FlatParams
    from unet_distributed_amd.utils.checkpoint import export_model
    cfg = Config(img_size=32, in_channels=4, dtype="fp32", checkpoint_dir=str(tmp_path))
    spec = spec_from_config(cfg)
    flat = FlatParams(spec)
    flat.load_dict(reference.init_params(spec, seed=3))
    d = export_model(cfg, spec, flat)
    # the GraphDef is the consumed artefact: no JSON side-car needed (sanity_check_trained_model.py:37-41)
    os.remove(os.path.join(d, "saved_model.json"))
    model = load_saved_model(d, device="cpu", batch=4)
    assert (model.spec.in_channels, model.spec.base, model.img_size) == (4, 32, 32)
    x, y = synthetic_brats(10, 32, 4, seed=1)
    p = model.predict(x)
    with torch.no_grad():
        ref = reference.forward(spec, flat.params(), torch.from_numpy(x), train=False, dropout=False)
    np.testing.assert_allclose(p, ref.numpy(), atol=1e-5)
    # reference batching quirk: range(0, n - bs, bs) -> n=10, bs=4 -> starts 0, 4
    assert sanity_check.batch_starts(10, 4) == [0, 4]
    assert sanity_check.batch_starts(8, 4) == [0]                  # last full batch dropped
    assert sanity_check.batch_starts(10, 4, all_batches=True) == [0, 4, 8]
    avg = sanity_check.main(["--export_dir", d, "--synthetic", "10", "--batch_size", "4", "--device", "cpu"])
    want = np.mean([sanity_dice(y[s:s + 4], p[s:s + 4]) for s in (0, 4)])
    assert abs(avg - want) < 1e-6
    assert "Average Dice for Test Set" in capsys.readouterr().out
