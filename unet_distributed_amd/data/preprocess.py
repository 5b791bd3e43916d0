"""BraTS 2016 (.mha) -> training ``.npy`` slices (`preprocess.py`, C20).

Behaviour of the reference's ``create_datasets_4`` (`preprocess.py:136-281`),
re-implemented as a streaming pass (no SimpleITK / OpenCV on this image):

* case folders are split train/test by position: every 5th case (index
  ``i % 5 == 0`` in the listing) is a test case (`preprocess.py:186-189`).  The
  reference iterates ``os.listdir`` order (filesystem dependent); we sort the
  listing so the split is reproducible -- pass ``sort=False`` for listdir order;
* inside a case, a sub-folder whose 5th dot-field is ``MR_<series>`` holds the
  T1 / T1c / Flair / T2 volume, any other ``.mha`` is the ground truth
  (`preprocess.py:33-55`); incomplete cases are still used, as in the reference;
* every volume is centre-cropped to ``img_rows x img_cols`` (lower margin
  ``floor((size-rows)/2)``, upper ``floor((size-rows+1)/2)``, `preprocess.py:
  118-122`), optionally shrunk by an integer factor, and z-scored per volume
  (`preprocess.py:130-134`);
* image channels are ``[T1c, T2, Flair, T1]`` -- the reference's tuple
  unpacking order (`preprocess.py:193,209-213`) -- and masks are the one-hot
  labels 1..4 (necrosis, edema, non-enhancing, enhancing);
* slices ``n`` (1-based) with ``n % slice_by == 0`` are kept; every other kept
  training slice is mirrored left-right (``cv2.flip(img, 1)``,
  `preprocess.py:239-244`);
* outputs ``imgs_train.npy``, ``msks_train.npy``, ``imgs_test.npy``,
  ``msks_test.npy`` in NHWC.  [Deviation] written as float32 (the reference
  writes float64 then every consumer casts to float32, `preprocess.py:300-301`)
  and filled through ``np.lib.format.open_memmap`` so the host never holds the
  whole dataset.
"""

import os
import time
from typing import List, Optional, Tuple

import numpy as np

from .mha import MetaImage, read_mha

SERIES = ("T1", "T1c", "Flair", "T2")


def find_case_files(case_dir: str) -> Tuple[dict, Optional[str], bool]:
    files, truth = {}, None
    for sub in sorted(os.listdir(case_dir)):
        sub_path = os.path.join(case_dir, sub)
        if not os.path.isdir(sub_path):
            continue
        for fn in sorted(os.listdir(sub_path)):
            if os.path.splitext(fn)[1] != ".mha":
                continue
            parts = sub.split(".")
            protocol_series = parts[4] if len(parts) > 4 else ""
            protocol = protocol_series.split("_")[0]
            if protocol == "MR":
                series = protocol_series.split("_")[1] if "_" in protocol_series else ""
                if series in SERIES:
                    files[series] = os.path.join(sub_path, fn)
            else:
                truth = os.path.join(sub_path, fn)
    complete = all(s in files for s in SERIES) and truth is not None
    return files, truth, complete


def crop_shrink(img: np.ndarray, rows: int, cols: int, factor: int = 1) -> np.ndarray:
    """``sitk.Crop`` to rows x cols in-plane (x = last array axis gets ``rows``
    like the reference's (x, y) size order) then ``sitk.Shrink`` by ``factor``."""
    z, y, x = img.shape
    lx, ux = (x - rows) // 2, (x - rows + 1) // 2
    ly, uy = (y - cols) // 2, (y - cols + 1) // 2
    out = img[:, ly:y - uy, lx:x - ux]
    if factor != 1:
        o = (factor - 1) // 2
        out = out[:, o::factor, o::factor]
    return out


def normalize(a: np.ndarray) -> np.ndarray:
    a = a.astype(np.float64)
    return (a - a.mean()) / a.std()


def _load(path: Optional[str], like: Optional[np.ndarray]) -> np.ndarray:
    if path is None:
        if like is None:
            raise IOError("case has no readable volumes")
        return np.zeros_like(like)          # the reference substitutes an empty sitk.Image
    return read_mha(path).array


def case_arrays(case_dir: str, rows: int, cols: int, factor: int = 1):
    files, truth, complete = find_case_files(case_dir)
    first = next((files[s] for s in SERIES if s in files), None)
    ref = read_mha(first).array if first else None
    vols = {s: crop_shrink(_load(files.get(s), ref), rows, cols, factor) for s in SERIES}
    msk = crop_shrink(_load(truth, ref), rows, cols, factor)
    img = np.stack([normalize(vols["T1c"]), normalize(vols["T2"]), normalize(vols["Flair"]),
                    normalize(vols["T1"])], axis=-1).astype(np.float32)
    lab = np.stack([(msk == k) for k in (1, 2, 3, 4)], axis=-1).astype(np.float32)
    return img, lab, complete


def create_datasets(img_path: str, out_path: str, img_rows: int = 128, img_cols: int = 128,
                    slice_by: int = 5, resize_factor: int = 1, sort: bool = True, verbose: bool = True):
    t0 = time.time()
    names = os.listdir(img_path)
    if sort:
        names = sorted(names)
    cases: List[Tuple[str, bool]] = []
    for i, n in enumerate(names):
        d = os.path.join(img_path, n)
        if os.path.isdir(d):
            cases.append((d, i % 5 != 0))
    # pass 1: slice counts (volume depth from the header only)
    depth = {}
    for d, _ in cases:
        files, truth, _ = find_case_files(d)
        p = next((files[s] for s in SERIES if s in files), truth)
        depth[d] = read_mha(p).array.shape[0] if p else 0
    n_tr = sum(depth[d] // slice_by for d, tr in cases if tr)
    n_te = sum(depth[d] // slice_by for d, tr in cases if not tr)
    _, r, c = crop_shrink(np.zeros((1, img_cols, img_rows), np.uint8), img_rows, img_cols, resize_factor).shape
    os.makedirs(out_path, exist_ok=True)
    mm = np.lib.format.open_memmap
    tr_i = mm(os.path.join(out_path, "imgs_train.npy"), "w+", np.float32, (n_tr, r, c, 4))
    tr_m = mm(os.path.join(out_path, "msks_train.npy"), "w+", np.float32, (n_tr, r, c, 4))
    te_i = mm(os.path.join(out_path, "imgs_test.npy"), "w+", np.float32, (n_te, r, c, 4))
    te_m = mm(os.path.join(out_path, "msks_test.npy"), "w+", np.float32, (n_te, r, c, 4))
    ktr = kte = 0
    for ci, (d, is_tr) in enumerate(cases):
        img, lab, complete = case_arrays(d, img_rows, img_cols, resize_factor)
        if verbose:
            print(ci, "Train:", is_tr, "complete:", complete, os.path.basename(d), flush=True)
        for s in range(img.shape[0]):
            if (s + 1) % slice_by:
                continue
            if is_tr:
                if ktr % 2 == 0:
                    tr_i[ktr], tr_m[ktr] = img[s], lab[s]
                else:                         # cv2.flip(img, 1): mirror the columns
                    tr_i[ktr], tr_m[ktr] = img[s][:, ::-1], lab[s][:, ::-1]
                ktr += 1
            else:
                te_i[kte], te_m[kte] = img[s], lab[s]
                kte += 1
    for a in (tr_i, tr_m, te_i, te_m):
        a.flush()
    if verbose:
        print("Saving to .npy files done.")
        print("Train ", ktr)
        print("Test  ", kte)
        print("Done in", time.time() - t0)
    return ktr, kte


def main(argv=None):
    import argparse
    from .. import settings
    p = argparse.ArgumentParser(description="BraTS .mha volumes -> .npy training slices")
    p.add_argument("--data_path", default=settings.DATA_PATH)
    p.add_argument("--out_path", default=settings.OUT_PATH)
    p.add_argument("--img_rows", type=int, default=settings.IMG_ROWS)
    p.add_argument("--img_cols", type=int, default=settings.IMG_COLS)
    p.add_argument("--slice_by", type=int, default=settings.SLICE_BY)
    p.add_argument("--rescale_factor", type=int, default=settings.RESCALE_FACTOR)
    p.add_argument("--listdir_order", action="store_true", help="split on os.listdir order like the reference")
    a = p.parse_args(argv)
    create_datasets(a.data_path, a.out_path, a.img_rows, a.img_cols, a.slice_by, a.rescale_factor,
                    sort=not a.listdir_order)


if __name__ == "__main__":
    main()
