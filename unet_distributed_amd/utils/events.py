"""TensorBoard event files without TensorFlow/tensorboard installed.

Reproduces the reference's summaries (`test_dist.py:275-298`, `322-326`):
scalars and histograms of loss / dice / sensitivity / specificity,
``percent_complete``, the ``*_test`` scalars, and up to TENSORBOARD_IMAGES
images of predictions / ground_truth / images (`settings_dist.py:42`).

Files are TFRecord-framed ``Event`` protos (length, masked CRC32C of the
length, payload, masked CRC32C of the payload), hand-encoded in protobuf wire
format; images are encoded as grayscale PNG with zlib.
"""

import os
import socket
import struct
import time
import zlib

import numpy as np

from .tf_bundle import _fbytes, _field, _fv, crc32c, mask_crc


def _fdouble(num, v):
    return _field(num, 1, struct.pack("<d", float(v)))


def _ffloat(num, v):
    return _field(num, 5, struct.pack("<f", float(v)))


def png_gray(img: np.ndarray) -> bytes:
    """uint8 [H, W] -> PNG bytes."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    raw = b"".join(b"\x00" + img[r].tobytes() for r in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "ab")
        self._write_event(_fdouble(1, time.time()) + _fbytes(3, b"brain.Event:2"))

    def _write_record(self, data: bytes):
        ln = struct.pack("<Q", len(data))
        self.f.write(ln + struct.pack("<I", mask_crc(crc32c(ln))) + data
                     + struct.pack("<I", mask_crc(crc32c(data))))

    def _write_event(self, payload: bytes):
        self._write_record(payload)

    def _summary(self, step: int, values: bytes):
        self._write_event(_fdouble(1, time.time()) + _fv(2, int(step)) + _fbytes(5, values))

    def scalars(self, step: int, d: dict):
        vals = b"".join(_fbytes(1, _fbytes(1, k.encode()) + _ffloat(2, v)) for k, v in d.items())
        self._summary(step, vals)

    def histogram(self, step: int, tag: str, values):
        a = np.asarray(values, dtype=np.float64).reshape(-1)
        if a.size == 0:
            return
        lo, hi = float(a.min()), float(a.max())
        edges = np.linspace(lo, hi if hi > lo else lo + 1e-12, 31)[1:]
        counts = np.histogram(a, bins=np.concatenate([[lo - 1e-12], edges]))[0].astype(np.float64)
        packed_l = b"".join(struct.pack("<d", x) for x in edges)
        packed_c = b"".join(struct.pack("<d", x) for x in counts)
        h = (_fdouble(1, lo) + _fdouble(2, hi) + _fdouble(3, a.size) + _fdouble(4, a.sum())
             + _fdouble(5, (a * a).sum()) + _fbytes(6, packed_l) + _fbytes(7, packed_c))
        self._summary(step, _fbytes(1, _fbytes(1, tag.encode()) + _fbytes(5, h)))

    def images(self, step: int, tag: str, batch: np.ndarray, max_outputs: int = 3):
        """batch: [N, H, W] or [N, H, W, C] float; the first channel is shown."""
        b = np.asarray(batch, dtype=np.float32)
        if b.ndim == 4:
            b = b[..., 0]
        vals = b""
        for i in range(min(max_outputs, b.shape[0])):
            x = b[i]
            lo, hi = float(x.min()), float(x.max())
            u8 = ((x - lo) / (hi - lo + 1e-12) * 255.0).astype(np.uint8)
            img = _fv(1, u8.shape[0]) + _fv(2, u8.shape[1]) + _fv(3, 1) + _fbytes(4, png_gray(u8))
            t = "%s/image/%d" % (tag, i) if max_outputs > 1 else "%s/image" % tag
            vals += _fbytes(1, _fbytes(1, t.encode()) + _fbytes(4, img))
        if vals:
            self._summary(step, vals)

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


def read_events(path: str):
    """Parse an event file back (used by tests): list of (step, {tag: value})."""
    from .tf_bundle import _parse
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        (n,) = struct.unpack("<Q", data[pos:pos + 8])
        (lc,) = struct.unpack("<I", data[pos + 8:pos + 12])
        if mask_crc(crc32c(data[pos:pos + 8])) != lc:
            raise IOError("bad length crc")
        payload = data[pos + 12:pos + 12 + n]
        (dc,) = struct.unpack("<I", data[pos + 12 + n:pos + 16 + n])
        if mask_crc(crc32c(payload)) != dc:
            raise IOError("bad data crc")
        pos += 16 + n
        ev = _parse(payload)
        step = ev.get(2, [0])[0]
        vals = {}
        for s in ev.get(5, []):
            for v in _parse(s).get(1, []):
                pv = _parse(v)
                tag = pv[1][0].decode()
                if 2 in pv:
                    vals[tag] = struct.unpack("<f", pv[2][0])[0]
                else:
                    vals[tag] = None
        out.append((step, vals))
    return out
