"""Flag surface (reference names/defaults + absl bool forms), data pipeline (CPU)."""
import numpy as np
import pytest

from unet_distributed_amd.config import parse_args
from unet_distributed_amd.data import datasets


def test_reference_flag_defaults():
    c = parse_args([])
    assert c.const_learningrate is True and c.learning_rate == 0.0005 and c.lr_fraction == 0.2
    assert c.decay_steps == 100 and c.is_sync == 1 and c.batch_size == 1024 and c.epochs == 10
    assert c.use_upsampling is False


@pytest.mark.parametrize("argv,val", [(["--use_upsampling"], True), (["--use_upsampling=True"], True),
                                      (["--use_upsampling=false"], False), (["--nouse_upsampling"], False),
                                      (["--use_upsampling", "1"], True)])
def test_absl_style_booleans(argv, val):
    assert parse_args(argv).use_upsampling is val


def test_readme_aliases_and_ext_flags():
    c = parse_args(["--learningrate", "0.001", "--num_threads", "8", "--dtype", "fp16", "--norm", "group",
                    "--dims", "3", "--in_channels", "4", "--loss", "dice_bce", "--synthetic"])
    assert c.learning_rate == 0.001 and c.num_threads == 8 and c.dtype == "fp16" and c.norm == "group"
    assert c.dims == 3 and c.in_channels == 4 and c.loss == "dice_bce" and c.synthetic


def test_unknown_flag_rejected():
    with pytest.raises(SystemExit):
        parse_args(["--not_a_flag", "1"])


def test_synthetic_deterministic_and_shaped():
    a = datasets.synthetic_brats(4, 32, 4, seed=3)
    b = datasets.synthetic_brats(4, 32, 4, seed=3)
    assert a[0].shape == (4, 32, 32, 4) and a[1].shape == (4, 32, 32, 1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert set(np.unique(a[1])) <= {0.0, 1.0}
    x3, y3 = datasets.synthetic_brats(2, 16, 4, dims=3, seed=1)
    assert x3.shape == (2, 16, 16, 16, 4)


def test_update_channels_modes():
    rng = np.random.default_rng(0)
    imgs = rng.random((3, 8, 8, 4)).astype(np.float64)
    msks = (rng.random((3, 8, 8, 4)) > 0.8).astype(np.float64)
    i1, m1 = datasets.update_channels(imgs, msks, 1, 1, 1)
    assert np.allclose(i1[..., 0], imgs[..., 2]) and np.allclose(m1[..., 0], msks.sum(-1))
    i2, m2 = datasets.update_channels(imgs, msks, 1, 1, 2)
    assert np.allclose(i2[..., 0], imgs[..., 0]) and np.allclose(m2[..., 0], msks[..., 3])
    i3, m3 = datasets.update_channels(imgs, msks, 1, 1, 3)
    assert np.allclose(m3[..., 0], msks[..., 0] + msks[..., 2] + msks[..., 3])
    i4, _ = datasets.update_channels(imgs, msks, 4, 1, 4)
    assert np.allclose(i4, imgs) and i4.dtype == np.float32


def test_epoch_sampler_partitions_global_batches():
    n, gb, world = 100, 16, 4
    shards = [datasets.EpochSampler(n, gb, r, world, seed=7).epoch_indices(2) for r in range(world)]
    assert all(s.shape == (6, 4) for s in shards)
    allidx = np.concatenate([s.reshape(-1) for s in shards])
    assert len(set(allidx.tolist())) == len(allidx) == 96          # disjoint, truncated to whole batches
    s2 = datasets.EpochSampler(n, gb, 0, world, seed=7).epoch_indices(3)
    assert not np.array_equal(s2, shards[0])                         # reshuffled each epoch


def test_loader_matches_direct_indexing():
    from unet_distributed_amd.data.loader import BatchLoader
    x, y = datasets.synthetic_brats(20, 16, 4, seed=0)
    idx = np.array([5, 1, 7, 3])
    ld = BatchLoader(x, y, per_rank=4, threads=2)
    bx, by = ld.gather(idx)
    assert np.array_equal(bx.numpy(), x[np.sort(idx)]) and np.array_equal(by.numpy(), y[np.sort(idx)])
