"""MetaImage (.mha / .mhd) volumes without SimpleITK.

The reference reads BraTS volumes with ``sitk.ReadImage`` (`preprocess.py:
80-115`); SimpleITK is not available on the MI355X image, so this is a small
self-contained reader/writer for the subset BraTS uses: an ASCII
``Key = Value`` header, ``ElementDataFile = LOCAL`` (data appended to the
header) or a detached raw file, optional zlib ``CompressedData``, any
``MET_*`` scalar element type, either byte order.

Arrays are returned in ``sitk.GetArrayFromImage`` order, i.e. the header's
``DimSize`` reversed: (z, y, x) for a 3-D volume.
"""

import os
import zlib
from typing import Dict, Tuple

import numpy as np

_MET = {
    "MET_CHAR": np.int8, "MET_UCHAR": np.uint8, "MET_SHORT": np.int16, "MET_USHORT": np.uint16,
    "MET_INT": np.int32, "MET_UINT": np.uint32, "MET_LONG": np.int32, "MET_ULONG": np.uint32,
    "MET_LONG_LONG": np.int64, "MET_ULONG_LONG": np.uint64, "MET_FLOAT": np.float32,
    "MET_DOUBLE": np.float64,
}
_MET_INV = {np.dtype(v): k for k, v in reversed(list(_MET.items()))}


class MetaImage:
    def __init__(self, array: np.ndarray, spacing=None, origin=None, header=None):
        self.array = array
        nd = array.ndim
        self.spacing = tuple(spacing) if spacing is not None else (1.0,) * nd
        self.origin = tuple(origin) if origin is not None else (0.0,) * nd
        self.header = header or {}

    def GetSize(self) -> Tuple[int, ...]:      # sitk convention: (x, y, z)
        return tuple(reversed(self.array.shape))


def _parse_header(f) -> Tuple[Dict[str, str], int]:
    hdr = {}
    while True:
        line = f.readline()
        if not line:
            break
        text = line.decode("latin-1").strip()
        if "=" not in text:
            continue
        k, v = text.split("=", 1)
        k, v = k.strip(), v.strip()
        hdr[k] = v
        if k == "ElementDataFile":
            break
    return hdr, f.tell()


def read_mha(path: str) -> MetaImage:
    with open(path, "rb") as f:
        hdr, data_off = _parse_header(f)
        dims = [int(d) for d in hdr["DimSize"].split()]
        nch = int(hdr.get("ElementNumberOfChannels", "1"))
        dt = np.dtype(_MET[hdr["ElementType"]])
        msb = hdr.get("BinaryDataByteOrderMSB", hdr.get("ElementByteOrderMSB", "False")).lower() == "true"
        dt = dt.newbyteorder(">" if msb else "<")
        src = hdr["ElementDataFile"]
        if src == "LOCAL":
            f.seek(data_off)
            raw = f.read()
        else:
            with open(os.path.join(os.path.dirname(path), src), "rb") as g:
                raw = g.read()
    if hdr.get("CompressedData", "False").lower() == "true":
        raw = zlib.decompress(raw)
    count = int(np.prod(dims)) * nch
    arr = np.frombuffer(raw, dtype=dt, count=count).astype(dt.newbyteorder("="))
    shape = tuple(reversed(dims)) + ((nch,) if nch > 1 else ())
    spacing = [float(s) for s in hdr.get("ElementSpacing", " ".join(["1"] * len(dims))).split()]
    origin = [float(s) for s in hdr.get("Offset", hdr.get("Origin", " ".join(["0"] * len(dims)))).split()]
    return MetaImage(arr.reshape(shape), spacing, origin, hdr)


def write_mha(path: str, array: np.ndarray, spacing=None, origin=None, compress: bool = False) -> None:
    a = np.ascontiguousarray(array)
    et = _MET_INV[a.dtype.newbyteorder("=") if a.dtype.byteorder not in "=|" else a.dtype]
    dims = list(reversed(a.shape))
    raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
    if compress:
        raw = zlib.compress(raw)
    lines = ["ObjectType = Image", "NDims = %d" % a.ndim, "BinaryData = True",
             "BinaryDataByteOrderMSB = False", "CompressedData = %s" % ("True" if compress else "False")]
    if compress:
        lines.append("CompressedDataSize = %d" % len(raw))
    lines += ["Offset = " + " ".join(str(o) for o in (origin or [0] * a.ndim)),
              "ElementSpacing = " + " ".join(str(s) for s in (spacing or [1] * a.ndim)),
              "DimSize = " + " ".join(str(d) for d in dims),
              "ElementType = " + et, "ElementDataFile = LOCAL"]
    with open(path, "wb") as f:
        f.write(("\n".join(lines) + "\n").encode("latin-1"))
        f.write(raw)
