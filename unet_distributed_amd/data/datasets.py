"""Datasets: reference .npy slices, channel/mode selection, synthetic BraTS data.

* ``load_data`` / ``update_channels`` reproduce `preprocess.py:281-350`
  (memory-mapped ``imgs_{train,test}.npy`` / ``msks_*.npy``; MODE 1 FLAIR ->
  whole tumour, MODE 2 T1c -> enhancing, MODE 3 T2 -> core).  Quirk fixes:
  float32 instead of float64 (Q14), and an explicit MODE 4 [EXT] that keeps
  all four modalities (the reference zero-fills images for any other mode, Q13).
* ``synthetic_brats`` generates BraTS-shaped slices (z-scored multi-modal
  images with elliptical "tumours" and their masks) deterministically from a
  seed, so training can run -- and Dice can actually improve -- without the
  private BraTS data (README.md:36-47).
* ``EpochSampler`` replaces ``get_epoch`` (`data.py:29-54`): one shuffle per
  epoch from a seed SHARED by all ranks (the reference's unseeded per-worker
  shuffles overlap, Q10), truncation to whole global batches, and per-rank
  contiguous shards of each global batch (`test_dist.py:385-394`).
"""

import os
from typing import Tuple

import numpy as np


def load_data(data_path: str, prefix: str = "_train"):
    imgs = np.load(os.path.join(data_path, "imgs" + prefix + ".npy"), mmap_mode="r", allow_pickle=False)
    msks = np.load(os.path.join(data_path, "msks" + prefix + ".npy"), mmap_mode="r", allow_pickle=False)
    return imgs, msks


def update_channels(imgs, msks, input_no=1, output_no=1, mode=1):
    """Channel-last selection (`preprocess.py:287-350`), returns float32 arrays."""
    shp = imgs.shape
    new_imgs = np.zeros((shp[0], shp[1], shp[2], input_no), dtype=np.float32)
    new_msks = np.zeros((shp[0], shp[1], shp[2], output_no), dtype=np.float32)
    if mode == 1:
        new_imgs[..., 0] = imgs[..., 2]                                     # FLAIR
        new_msks[..., 0] = msks[..., 0] + msks[..., 1] + msks[..., 2] + msks[..., 3]
    elif mode == 2:
        new_imgs[..., 0] = imgs[..., 0]                                     # T1 post
        new_msks[..., 0] = msks[..., 3]
    elif mode == 3:
        new_imgs[..., 0] = imgs[..., 1]                                     # T2
        new_msks[..., 0] = msks[..., 0] + msks[..., 2] + msks[..., 3]
    elif mode == 4:                                                          # [EXT] all modalities
        k = min(input_no, shp[3])
        new_imgs[..., :k] = imgs[..., :k]
        new_msks[..., 0] = msks[..., 0] + msks[..., 1] + msks[..., 2] + msks[..., 3]
    else:
        new_msks[..., 0] = msks[..., 0] + msks[..., 1] + msks[..., 2] + msks[..., 3]
    return new_imgs, new_msks


def synthetic_brats(n: int, img: int = 128, channels: int = 4, dims: int = 2, seed: int = 0,
                    dtype=np.float32, difficulty: str = "easy") -> Tuple[np.ndarray, np.ndarray]:
    """Deterministic BraTS-like samples: [n, (img,) img, img, channels] images and
    [n, ..., 1] binary masks.  Each sample is a smooth 'brain' disc plus 0-2
    ellipsoidal lesions that are hyper-intense in a sample-dependent subset of
    the modalities, then z-scored per sample like `preprocess.py:117-124`.

    ``difficulty="hard"``: a segmentation task that does not saturate (its Dice
    plateau is in the reference's MODE-1 range, 0.78-0.80 on BraTS,
    `settings_dist.py:30`): 1-4 small lesions (3-7 px radius), each visible in only
    one or two modalities at low contrast (0.27-0.6 before noise, 0.7-1.5 sigma of the
    noise), sigma 0.4 noise, a smooth per-sample intensity bias field, and look-alike blobs that are
    bright in a single modality but are NOT lesions -- a lesion bright in one modality
    and a distractor differ only in shape / size statistics, so the errors at
    boundaries and on single-modality lesions remain."""
    if difficulty == "hard":
        return _synthetic_hard(n, img, channels, dims, seed, dtype)
    if difficulty != "easy":
        raise ValueError("synthetic difficulty must be easy or hard")
    rng = np.random.default_rng(seed)
    sp = (img,) * dims
    grids = np.meshgrid(*[np.linspace(-1, 1, img, dtype=np.float32)] * dims, indexing="ij")
    imgs = np.empty((n,) + sp + (channels,), dtype=dtype)
    msks = np.zeros((n,) + sp + (1,), dtype=dtype)
    r2 = sum(g * g for g in grids)
    brain = (r2 < 0.8).astype(np.float32)
    for i in range(n):
        x = np.repeat(brain[..., None], channels, axis=-1) * (0.6 + 0.2 * rng.random(channels, dtype=np.float32))
        m = np.zeros(sp, dtype=bool)
        for _ in range(rng.integers(0, 3)):
            c = rng.uniform(-0.5, 0.5, size=dims).astype(np.float32)
            ax = rng.uniform(0.08, 0.3, size=dims).astype(np.float32)
            e = sum(((g - cc) / a) ** 2 for g, cc, a in zip(grids, c, ax))
            m |= e < 1.0
        if m.any():
            gain = rng.uniform(0.5, 1.5, size=channels).astype(np.float32)
            x = x + m[..., None] * gain
        x = x + 0.15 * rng.standard_normal(x.shape).astype(np.float32)
        x = (x - x.mean()) / (x.std() + 1e-6)
        imgs[i] = x
        msks[i, ..., 0] = m
    return imgs, msks


def _synthetic_hard(n, img, channels, dims, seed, dtype):
    rng = np.random.default_rng((seed, 7))
    sp = (img,) * dims
    grids = np.meshgrid(*[np.linspace(-1, 1, img, dtype=np.float32)] * dims, indexing="ij")
    px = 2.0 / img                                     # one pixel in grid units
    imgs = np.empty((n,) + sp + (channels,), dtype=dtype)
    msks = np.zeros((n,) + sp + (1,), dtype=dtype)
    brain = (sum(g * g for g in grids) < 0.8).astype(np.float32)

    def blob(radius_px):
        c = rng.uniform(-0.55, 0.55, size=dims).astype(np.float32)
        ax = (radius_px * px * rng.uniform(0.7, 1.3, size=dims)).astype(np.float32)
        return sum(((g - cc) / a) ** 2 for g, cc, a in zip(grids, c, ax)) < 1.0

    for i in range(n):
        base = 0.6 + 0.2 * rng.random(channels, dtype=np.float32)
        bias = 1.0 + 0.25 * sum(rng.uniform(-1, 1) * g for g in grids)       # smooth bias field
        x = (brain * bias)[..., None] * base
        m = np.zeros(sp, dtype=bool)
        for _ in range(rng.integers(1, 5)):
            b = blob(rng.uniform(3.0, 7.0)) & (brain > 0)
            chans = rng.choice(channels, size=rng.integers(1, min(2, channels) + 1), replace=False)
            for ch in chans:
                x[..., ch] += b * rng.uniform(0.45, 1.0) * 0.6
            m |= b
        for _ in range(rng.integers(0, 3)):                   # single-modality look-alikes
            b = blob(rng.uniform(1.5, 4.0)) & (brain > 0) & ~m
            x[..., rng.integers(channels)] += b * rng.uniform(0.35, 0.9) * 0.5
        x = x + 0.4 * rng.standard_normal(x.shape).astype(np.float32)
        x = (x - x.mean()) / (x.std() + 1e-6)
        imgs[i] = x
        msks[i, ..., 0] = m
    return imgs, msks


class EpochSampler:
    """Shared-seed epoch shuffling and per-rank sharding of global batches."""

    def __init__(self, n: int, global_batch: int, rank: int, world: int, seed: int = 0):
        if global_batch % world:
            raise ValueError("global batch %d not divisible by world size %d" % (global_batch, world))
        self.n = n
        self.gb = global_batch
        self.rank = rank
        self.world = world
        self.seed = seed
        self.per_rank = global_batch // world
        self.num_batches = n // global_batch
        if self.num_batches == 0:
            raise ValueError("dataset of %d samples smaller than one global batch (%d)" % (n, global_batch))

    def epoch_indices(self, epoch: int) -> np.ndarray:
        perm = np.random.default_rng((self.seed, epoch)).permutation(self.n)
        perm = perm[: self.num_batches * self.gb].reshape(self.num_batches, self.gb)
        s = self.rank * self.per_rank
        return perm[:, s: s + self.per_rank]
