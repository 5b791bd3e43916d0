"""TensorFlow V2 tensor-bundle checkpoints, written and read without TensorFlow.

The reference saves with ``tf.train.Saver`` (`test_dist.py:269-271,446,490`)
through ``tf.train.Supervisor(save_model_secs=60)`` (`test_dist.py:347-355`):
``<prefix>.index`` + ``<prefix>.data-00000-of-00001`` plus a ``checkpoint``
text file naming the latest prefix.  We write that on-disk layout (the V2
bundle format TF tooling such as ``tf.train.NewCheckpointReader`` reads):

* ``.data-00000-of-00001``: the raw little-endian tensor bytes, back to back;
* ``.index``: a LevelDB-format SSTable (no compression) whose empty key maps to
  a ``BundleHeaderProto`` and every tensor name to a ``BundleEntryProto``
  (dtype, shape, shard 0, offset, size, masked CRC32C of the bytes);
* block trailers carry masked CRC32C of block contents + type byte; the footer
  ends with the table magic ``0xdb4775248b80fb57``.

Format parity is UNPINNED: TensorFlow is not installed here and the reference
ships no TF-written checkpoint, so the files are verified against the format's
structure (SSTable footer / block CRCs / BundleEntryProto fields) and by
round-trip, not by a TF reader.

Protobufs are hand-encoded (wire format) since TF's .proto files are absent.
CRC32C runs in the native runtime (SSE4.2), with a pure-Python fallback.
"""

import os
import struct
from typing import Dict, Tuple

import numpy as np

TABLE_MAGIC = 0xDB4775248B80FB57
_DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3, np.dtype("uint8"): 4,
       np.dtype("int16"): 5, np.dtype("int8"): 6, np.dtype("int64"): 9, np.dtype("bool"): 10,
       np.dtype("float16"): 19}
_DT_INV = {v: k for k, v in _DT.items()}
_DT_INV[14] = "bfloat16"

# --------------------------------------------------------------------------- crc32c
_TABLE = None


def _py_crc32c(data: bytes, crc: int = 0) -> int:
    global _TABLE
    if _TABLE is None:
        _TABLE = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
            _TABLE.append(c)
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def crc32c(data, crc: int = 0) -> int:
    try:
        from .. import native
        if native.available():
            return native.lib().crc32c(memoryview(data).cast("B"), crc)
    except Exception:
        pass
    return _py_crc32c(bytes(data), crc)


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    r = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# --------------------------------------------------------------------------- protobuf wire
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _field(num, wire, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _fv(num, v: int) -> bytes:
    return _field(num, 0, _varint(v))


def _fbytes(num, b: bytes) -> bytes:
    return _field(num, 2, _varint(len(b)) + b)


def _parse(buf: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = _read_varint(buf, pos)
        elif wire == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wire == 2:
            n, pos = _read_varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wire == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError("unsupported wire type %d" % wire)
        out.setdefault(num, []).append(v)
    return out


def _header_proto() -> bytes:
    version = _fv(1, 1)  # VersionDef.producer = 1
    return _fv(1, 1) + _fv(2, 0) + _fbytes(3, version)   # num_shards, LITTLE endian, version


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    shape_pb = b"".join(_fbytes(2, _fv(1, int(d))) for d in shape)
    return (_fv(1, dtype) + _fbytes(2, shape_pb) + _fv(3, 0) + _fv(4, offset) + _fv(5, size)
            + _field(6, 5, struct.pack("<I", crc)))


# --------------------------------------------------------------------------- SSTable
def _block(entries, restart_interval=16) -> bytes:
    out = bytearray()
    restarts = []
    last = b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _write_block(f, contents: bytes) -> Tuple[int, int]:
    off = f.tell()
    f.write(contents)
    trailer_type = b"\x00"
    f.write(trailer_type + struct.pack("<I", mask_crc(crc32c(contents + trailer_type))))
    return off, len(contents)


def _handle(off, size) -> bytes:
    return _varint(off) + _varint(size)


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """Write ``prefix.index`` / ``prefix.data-00000-of-00001`` atomically."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    names = sorted(tensors)
    entries = []
    tmp_data = prefix + ".data-00000-of-00001.tmp"
    with open(tmp_data, "wb") as f:
        off = 0
        for n in names:
            a = np.asarray(tensors[n])          # (ascontiguousarray would promote 0-d to 1-d)
            if not a.flags.c_contiguous:
                a = a.copy()
            if a.dtype not in _DT:
                raise TypeError("unsupported dtype %s for %s" % (a.dtype, n))
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            entries.append((n.encode(), _entry_proto(_DT[a.dtype], a.shape, off, len(raw),
                                                      mask_crc(crc32c(raw)))))
            off += len(raw)
    kv = [(b"", _header_proto())] + entries
    tmp_idx = prefix + ".index.tmp"
    with open(tmp_idx, "wb") as f:
        # data blocks of ~256 KiB like TF's table::Options default
        index_entries = []
        cur, cur_size = [], 0
        blocks = []
        for k, v in kv:
            cur.append((k, v))
            cur_size += len(k) + len(v) + 8
            if cur_size >= 262144:
                blocks.append(cur)
                cur, cur_size = [], 0
        if cur or not blocks:
            blocks.append(cur)
        for blk in blocks:
            off, size = _write_block(f, _block(blk))
            index_entries.append((blk[-1][0] if blk else b"", _handle(off, size)))
        meta_off, meta_size = _write_block(f, _block([]))
        idx_off, idx_size = _write_block(f, _block(index_entries, restart_interval=1))
        footer = _handle(meta_off, meta_size) + _handle(idx_off, idx_size)
        footer = footer + b"\x00" * (40 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
        f.write(footer)
    os.replace(tmp_data, prefix + ".data-00000-of-00001")
    os.replace(tmp_idx, prefix + ".index")


def _read_block_entries(buf: bytes, off: int, size: int, verify=True):
    contents = buf[off:off + size]
    if verify:
        t = buf[off + size:off + size + 1]
        (m,) = struct.unpack("<I", buf[off + size + 1:off + size + 5])
        if mask_crc(crc32c(contents + t)) != m:
            raise IOError("SSTable block checksum mismatch")
    (nr,) = struct.unpack("<I", contents[-4:])
    limit = len(contents) - 4 - 4 * nr
    pos = 0
    last = b""
    out = []
    while pos < limit:
        shared, pos = _read_varint(contents, pos)
        nshared, pos = _read_varint(contents, pos)
        vlen, pos = _read_varint(contents, pos)
        key = last[:shared] + contents[pos:pos + nshared]
        pos += nshared
        val = contents[pos:pos + vlen]
        pos += vlen
        out.append((key, val))
        last = key
    return out


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    with open(prefix + ".index", "rb") as f:
        buf = f.read()
    (magic,) = struct.unpack("<Q", buf[-8:])
    if magic != TABLE_MAGIC:
        raise IOError("not an SSTable: %s.index" % prefix)
    footer = buf[-48:]
    _, p = _read_varint(footer, 0)
    _, p = _read_varint(footer, p)
    idx_off, p = _read_varint(footer, p)
    idx_size, p = _read_varint(footer, p)
    entries = []
    for _, handle in _read_block_entries(buf, idx_off, idx_size, verify):
        off, q = _read_varint(handle, 0)
        size, _ = _read_varint(handle, q)
        entries.extend(_read_block_entries(buf, off, size, verify))
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        data = f.read()
    out = {}
    for k, v in entries:
        if k == b"":
            continue
        fields = _parse(v)
        dtype = fields.get(1, [1])[0]
        shape = []
        for dim in _parse(fields[2][0]).get(2, []) if 2 in fields else []:
            shape.append(_parse(dim).get(1, [0])[0])
        off = fields.get(4, [0])[0]
        size = fields.get(5, [0])[0]
        raw = data[off:off + size]
        if verify and 6 in fields:
            (m,) = struct.unpack("<I", fields[6][0])
            if mask_crc(crc32c(raw)) != m:
                raise IOError("tensor checksum mismatch for %s" % k.decode())
        dt = _DT_INV[dtype]
        if dt == "bfloat16":
            a = np.frombuffer(raw, dtype=np.uint16).astype(np.uint32) << 16
            a = a.view(np.float32)
        else:
            a = np.frombuffer(raw, dtype=np.dtype(dt).newbyteorder("<"))
        out[k.decode()] = a.reshape(shape).copy()
    return out


# --------------------------------------------------------------------------- checkpoint state file
def write_checkpoint_state(directory: str, latest: str, all_paths) -> None:
    lines = ['model_checkpoint_path: "%s"' % latest]
    lines += ['all_model_checkpoint_paths: "%s"' % p for p in all_paths]
    tmp = os.path.join(directory, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(directory, "checkpoint"))


def read_checkpoint_state(directory: str):
    path = os.path.join(directory, "checkpoint")
    if not os.path.exists(path):
        return None, []
    latest, all_paths = None, []
    for line in open(path):
        line = line.strip()
        if line.startswith("model_checkpoint_path:"):
            latest = line.split(":", 1)[1].strip().strip('"')
        elif line.startswith("all_model_checkpoint_paths:"):
            all_paths.append(line.split(":", 1)[1].strip().strip('"'))
    return latest, all_paths
