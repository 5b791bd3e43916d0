"""Post-hoc check of an exported model (`sanity_check_trained_model.py`, C22).

Loads ``<checkpoint_dir>/saved_model`` (:mod:`unet_distributed_amd.inference`),
runs it over the test set in batches of 128 and prints the average per-batch
Dice with the script's own smoothing ``2(sum(a*b)+1)/(sum(a+b)+1)``
(`sanity_check_trained_model.py:30-35`).

Batch iteration reproduces the reference exactly by default:
``range(0, n - batch_size, batch_size)`` -- which drops the last full batch
whenever ``n`` is a multiple of the batch size, and the partial tail
(`sanity_check_trained_model.py:51`).  ``--all_batches`` covers every sample
instead (fix).
"""

import argparse
import os
import sys
import time

import numpy as np

from . import settings
from .data import datasets
from .ops.losses import sanity_dice


def batch_starts(n: int, batch_size: int, all_batches: bool = False):
    if all_batches:
        return list(range(0, n, batch_size))
    return list(range(0, n - batch_size, batch_size))


def main(argv=None) -> float:
    p = argparse.ArgumentParser(description="Average test-set Dice of an exported model")
    p.add_argument("--export_dir", default=os.path.join(settings.CHECKPOINT_DIRECTORY, "saved_model"))
    p.add_argument("--data_path", default=settings.OUT_PATH)
    p.add_argument("--batch_size", type=int, default=128)
    p.add_argument("--in_channels", type=int, default=settings.IN_CHANNEL_NO)
    p.add_argument("--out_channels", type=int, default=settings.OUT_CHANNEL_NO)
    p.add_argument("--mode", type=int, default=settings.MODE)
    p.add_argument("--device", default=None)
    p.add_argument("--backend", default="auto", choices=["auto", "native", "torch"])
    p.add_argument("--all_batches", action="store_true")
    p.add_argument("--synthetic", type=int, default=0, metavar="N",
                   help="use N synthetic test slices instead of the .npy files")
    a = p.parse_args(argv)
    from .inference import load_saved_model
    print("Loading trained model from directory {}".format(a.export_dir))
    model = load_saved_model(a.export_dir, device=a.device, batch=a.batch_size, backend=a.backend)
    print('-' * 38)
    print('Loading and preprocessing test data...')
    print('-' * 38)
    if a.synthetic:
        x, y = datasets.synthetic_brats(a.synthetic, model.img_size, model.spec.in_channels, model.spec.dims, seed=1)
    else:
        xi, yi = datasets.load_data(a.data_path, "_test")
        x, y = datasets.update_channels(xi, yi, a.in_channels, a.out_channels, a.mode)
    dice, nb = 0.0, 0
    t0 = time.time()
    for s in batch_starts(len(x), a.batch_size, a.all_batches):
        xb = np.asarray(x[s:s + a.batch_size], dtype=np.float32)
        yb = np.asarray(y[s:s + a.batch_size], dtype=np.float32)
        pb = model.predict(xb)
        dice += sanity_dice(yb, pb)
        nb += 1
    dt = time.time() - t0
    avg = dice / nb if nb else float("nan")
    print("Average Dice for Test Set = {}".format(avg))
    print("({} batches, {} backend, {:.1f} images/sec)".format(nb, model.name, nb * a.batch_size / max(dt, 1e-9)))
    return avg


if __name__ == "__main__":
    main()
    sys.exit(0)
