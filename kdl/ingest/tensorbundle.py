"""TensorFlow TensorBundle (checkpoint) reader/writer without TensorFlow.

A SavedModel's ``variables/`` holds ``variables.index`` (a LevelDB SSTable:
key ``""`` -> BundleHeaderProto, every other key -> BundleEntryProto) and
``variables.data-SSSSS-of-NNNNN`` shards with the raw little-endian tensor bytes
(SURVEY.md §2.9.3). Reading uses the native parser in ``kdl._rt`` (block CRC
checks, snappy); a pure-Python parser is kept as a cross-check and fallback.
The writer exists to synthesise fixtures (no real TF artifact is reachable
offline).
"""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np

from ..serving import protos as P

MAGIC = 0xDB4775248B80FB57
_NP = {P.DT_FLOAT: np.float32, P.DT_DOUBLE: np.float64, P.DT_INT32: np.int32, P.DT_INT64: np.int64,
       P.DT_UINT8: np.uint8, P.DT_INT8: np.int8, P.DT_INT16: np.int16, P.DT_BOOL: np.bool_,
       P.DT_HALF: np.float16}


# ------------------------------------------------------------------ pure-python SSTable
def _varint(b: bytes, i: int) -> tuple[int, int]:
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        if not c & 0x80:
            return v, i
        s += 7


def _crc32c_py(data: bytes, crc: int = 0) -> int:
    table = _crc32c_py.table
    c = crc ^ 0xFFFFFFFF
    for x in data:
        c = table[(c ^ x) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _mk_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_crc32c_py.table = _mk_table()


def crc32c(data: bytes, crc: int = 0) -> int:
    try:
        from ..ops._lib import rt
        return rt().crc32c(data, crc)
    except Exception:
        return _crc32c_py(data, crc)


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _snappy_py(b: bytes) -> bytes:
    n, i = _varint(b, 0)
    out = bytearray()
    while i < len(b):
        tag = b[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(b[i:i + nb], "little")
                i += nb
            ln += 1
            out += b[i:i + ln]
            i += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | b[i]
            i += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = b[i] | (b[i + 1] << 8)
            i += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[i:i + 4], "little")
            i += 4
        start = len(out) - off
        for k in range(ln):
            out.append(out[start + k])
    assert len(out) == n, "snappy length mismatch"
    return bytes(out)


def _block(data: bytes, off: int, size: int, verify: bool) -> bytes:
    raw = data[off:off + size]
    typ = data[off + size]
    if verify:
        want = struct.unpack_from("<I", data, off + size + 1)[0]
        if mask_crc(_crc32c_py(data[off:off + size + 1])) != want:
            raise ValueError("sstable: block checksum mismatch")
    if typ == 0:
        return raw
    if typ == 1:
        return _snappy_py(raw)
    raise ValueError(f"sstable: unknown compression {typ}")


def _entries(blk: bytes) -> list[tuple[bytes, bytes]]:
    nres = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    limit = len(blk) - 4 - 4 * nres
    out, key, i = [], b"", 0
    while i < limit:
        shared, i = _varint(blk, i)
        nonshared, i = _varint(blk, i)
        vlen, i = _varint(blk, i)
        key = key[:shared] + blk[i:i + nonshared]
        i += nonshared
        out.append((key, blk[i:i + vlen]))
        i += vlen
    return out


def read_sstable_py(data: bytes, verify: bool = True) -> list[tuple[bytes, bytes]]:
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != MAGIC:
        raise ValueError("not an SSTable (bad magic)")
    f = len(data) - 48
    _, i = _varint(data, f)
    _, i = _varint(data, i)          # metaindex handle
    ioff, i = _varint(data, i)
    isz, i = _varint(data, i)
    out = []
    for _, h in _entries(_block(data, ioff, isz, verify)):
        off, j = _varint(h, 0)
        sz, _ = _varint(h, j)
        out.extend(_entries(_block(data, off, sz, verify)))
    return out


def read_sstable(data: bytes, verify: bool = True) -> list[tuple[bytes, bytes]]:
    try:
        from ..ops._lib import rt
        return rt().read_sstable(data, verify)
    except RuntimeError:
        return read_sstable_py(data, verify)


# ------------------------------------------------------------------ bundle reader
class TensorBundle:
    """Random access to the tensors of ``<prefix>.index`` / ``<prefix>.data-*``."""

    def __init__(self, prefix: str | Path, verify: bool = True):
        self.prefix = str(prefix)
        kv = read_sstable(Path(self.prefix + ".index").read_bytes(), verify)
        self.header = None
        self.entries: dict[str, object] = {}
        for k, v in kv:
            if k == b"":
                self.header = P.BundleHeaderProto.FromString(v)
            else:
                self.entries[k.decode()] = P.BundleEntryProto.FromString(v)
        if self.header is None:
            raise ValueError("TensorBundle index has no header entry")
        if self.header.endianness != 0:
            raise ValueError("big-endian TensorBundle not supported")
        self.num_shards = max(1, self.header.num_shards)
        self._shards: dict[int, np.memmap] = {}
        self.verify = verify

    def _shard(self, i: int) -> np.memmap:
        if i not in self._shards:
            path = f"{self.prefix}.data-{i:05d}-of-{self.num_shards:05d}"
            self._shards[i] = np.memmap(path, dtype=np.uint8, mode="r")
        return self._shards[i]

    def keys(self) -> list[str]:
        return sorted(self.entries)

    def raw(self, key: str) -> bytes:
        e = self.entries[key]
        sh = self._shard(e.shard_id)
        return bytes(sh[e.offset:e.offset + e.size])

    def get(self, key: str) -> np.ndarray:
        e = self.entries[key]
        buf = self.raw(key)
        if self.verify and e.crc32c and crc32c(buf) != e.crc32c and mask_crc(crc32c(buf)) != e.crc32c:
            raise ValueError(f"tensor {key}: crc32c mismatch")
        if e.dtype == P.DT_STRING:
            return np.frombuffer(buf, dtype=np.uint8)
        if e.dtype not in _NP:
            raise TypeError(f"tensor {key}: unsupported dtype {e.dtype}")
        shape = tuple(d.size for d in e.shape.dim)
        return np.frombuffer(buf, dtype=_NP[e.dtype]).reshape(shape)


# ------------------------------------------------------------------ writer (fixtures)
def _put_varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _snappy_literal(raw: bytes) -> bytes:
    """Valid snappy stream made of literals (exercises the decoder's framing)."""
    out = bytearray(_put_varint(len(raw)))
    i = 0
    while i < len(raw):
        chunk = raw[i:i + 65536]
        ln = len(chunk) - 1
        if ln < 60:
            out.append(ln << 2)
        else:
            nb = (ln.bit_length() + 7) // 8
            out.append((59 + nb) << 2)
            out += ln.to_bytes(nb, "little")
        out += chunk
        i += len(chunk)
    return bytes(out)


def write_sstable(entries: list[tuple[bytes, bytes]], compress: bool = False, block_size: int = 4096,
                  restart_interval: int = 16) -> bytes:
    entries = sorted(entries)
    out = bytearray()
    index = []

    def flush(block_entries):
        buf, restarts, prev = bytearray(), [], b""
        for n, (k, v) in enumerate(block_entries):
            if n % restart_interval == 0:
                restarts.append(len(buf))
                shared = 0
            else:
                shared = 0
                while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                    shared += 1
            buf += _put_varint(shared) + _put_varint(len(k) - shared) + _put_varint(len(v))
            buf += k[shared:] + v
            prev = k
        for r in restarts or [0]:
            buf += struct.pack("<I", r)
        buf += struct.pack("<I", len(restarts or [0]))
        payload, typ = bytes(buf), 0
        if compress:
            payload, typ = _snappy_literal(payload), 1
        off = len(out)
        out.extend(payload)
        out.append(typ)
        out.extend(struct.pack("<I", mask_crc(_crc32c_py(payload + bytes([typ])))))
        return off, len(payload)

    cur, size = [], 0
    for k, v in entries:
        cur.append((k, v))
        size += len(k) + len(v)
        if size >= block_size:
            off, sz = flush(cur)
            index.append((cur[-1][0], _put_varint(off) + _put_varint(sz)))
            cur, size = [], 0
    if cur:
        off, sz = flush(cur)
        index.append((cur[-1][0], _put_varint(off) + _put_varint(sz)))
    meta_off, meta_sz = flush([])
    idx_off, idx_sz = flush(index)
    footer = _put_varint(meta_off) + _put_varint(meta_sz) + _put_varint(idx_off) + _put_varint(idx_sz)
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
    out += footer
    return bytes(out)


def write_bundle(prefix: str | Path, tensors: dict[str, np.ndarray], compress: bool = False,
                 extra_entries: dict[str, bytes] | None = None) -> None:
    """Write ``<prefix>.index`` + ``<prefix>.data-00000-of-00001``.

    ``extra_entries`` are raw string tensors (e.g. _CHECKPOINTABLE_OBJECT_GRAPH)."""
    prefix = str(prefix)
    Path(prefix).parent.mkdir(parents=True, exist_ok=True)
    data = bytearray()
    kv = [(b"", P.BundleHeaderProto(num_shards=1, endianness=0).SerializeToString())]
    inv = {np.dtype(v): k for k, v in _NP.items()}
    items = {k: np.ascontiguousarray(v) for k, v in tensors.items()}
    for key in sorted(items):
        a = items[key]
        raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
        e = P.BundleEntryProto(dtype=inv[a.dtype], shard_id=0, offset=len(data), size=len(raw),
                               crc32c=mask_crc(crc32c(raw)))
        for d in a.shape:
            e.shape.dim.add(size=int(d))
        data += raw
        kv.append((key.encode(), e.SerializeToString()))
    for key, raw in (extra_entries or {}).items():
        # TF stores string tensors as varint lengths + bytes; a 0-d string tensor
        e = P.BundleEntryProto(dtype=P.DT_STRING, shard_id=0, offset=len(data), size=len(raw))
        data += raw
        kv.append((key.encode(), e.SerializeToString()))
    Path(prefix + ".index").write_bytes(write_sstable(kv, compress=compress))
    Path(prefix + ".data-00000-of-00001").write_bytes(bytes(data))
