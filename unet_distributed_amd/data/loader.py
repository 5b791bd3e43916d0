"""Host batch loader: gathers a per-rank shard's samples into a (pinned) staging
buffer with the native multi-threaded row gather (``_C.gather_rows``), falling
back to numpy fancy indexing when the extension is unavailable.

Replaces the reference's full in-memory epoch materialisation (`data.py:29-54`
builds the whole shuffled epoch array every epoch): only the current batch is
copied, straight from the memory-mapped ``.npy`` arrays, with index order sorted
for sequential reads.  ``--num_threads`` (README.md:63) sizes the gather pool.
"""

import numpy as np
import torch


class BatchLoader:
    def __init__(self, x: np.ndarray, y: np.ndarray, per_rank: int, threads: int = 8, pin: bool = False):
        self.x, self.y = x, y
        self.threads = max(1, int(threads))
        self.bx = torch.empty((per_rank,) + tuple(x.shape[1:]), dtype=torch.float32, pin_memory=pin)
        self.by = torch.empty((per_rank,) + tuple(y.shape[1:]), dtype=torch.float32, pin_memory=pin)
        self._native = None
        try:
            from .. import native
            if native.available():
                self._native = native.lib()
        except Exception:
            self._native = None

    def _gather(self, src: np.ndarray, idx: np.ndarray, dst: torch.Tensor):
        n = len(idx)
        if (self._native is not None and src.dtype == np.float32 and src.flags.c_contiguous
                and dst.is_contiguous()):
            row = int(np.prod(src.shape[1:])) * 4
            ii = np.ascontiguousarray(idx, dtype=np.int64)
            self._native.gather_rows(src.ctypes.data, ii.ctypes.data, n, row, dst.data_ptr(), self.threads)
        else:
            dst.numpy()[:n] = src[idx]

    def gather(self, idx: np.ndarray):
        idx = np.sort(np.asarray(idx))
        self._gather(self.x, idx, self.bx)
        self._gather(self.y, idx, self.by)
        return self.bx, self.by
