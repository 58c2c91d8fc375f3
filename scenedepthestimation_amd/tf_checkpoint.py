"""TF1 tensor-bundle checkpoint reader (no TensorFlow needed).

The reference restores the MC-CNN branch with ``tf.train.Saver().restore(sess,
checkpoint)`` (process_functional.py:24-33) from a prefix such as
``./check_points_11_11/model_epoch14.ckpt`` (match_single.py:47, match.py:69);
the variables are ``conv{k}/weights`` (HWIO) and ``conv{k}/biases``
(mc_cnn_brunch.py:70-92).  A Saver V2 checkpoint (the TF1 default) is

* ``<prefix>.index``: a LevelDB-format sorted string table mapping tensor names to
  ``BundleEntryProto`` records (the empty key holds the ``BundleHeaderProto``);
* ``<prefix>.data-SSSSS-of-NNNNN``: the raw little-endian tensor bytes, located by
  (shard_id, offset, size) and checked by a masked CRC-32C.

This module restates those published formats directly: the table footer
(metaindex + index block handles, magic 0xdb4775248b80fb57), prefix-compressed
block entries with restart arrays, the 5-byte block trailer (compression type +
masked CRC-32C), and the protobuf wire encoding of the two records.  Only
uncompressed tables are accepted (what TF's bundle writer produces); a snappy
block raises ValueError.  Host-side file I/O only -- nothing here touches the GPU.
"""
from __future__ import annotations

import os
import struct

import numpy as np

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_LEN = 48
BLOCK_TRAILER_LEN = 5

# tensorflow/core/framework/types.proto DataType -> numpy
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DT_BFLOAT16 = 14

# ---------------------------------------------------------------------------
# CRC-32C (Castagnoli, reflected polynomial 0x82F63B78) and TF/LevelDB masking
# ---------------------------------------------------------------------------
_CRC_TABLE = None


def _crc_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        t = np.zeros((8, 256), np.uint32)
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            t[0, i] = c
        for k in range(1, 8):          # slicing-by-8 tables
            for i in range(256):
                c = int(t[k - 1, i])
                t[k, i] = (c >> 8) ^ int(t[0, c & 0xFF])
        _CRC_TABLE = [[int(v) for v in row] for row in t]
    return _CRC_TABLE


def crc32c(data, crc: int = 0) -> int:
    """CRC-32C of `data` (check value: crc32c(b"123456789") == 0xE3069283)."""
    t = _crc_table()
    t0, t1, t2, t3, t4, t5, t6, t7 = t
    mv = memoryview(bytes(data))
    c = crc ^ 0xFFFFFFFF
    n8 = len(mv) // 8 * 8
    words = struct.unpack_from("<%dQ" % (n8 // 8), mv, 0) if n8 else ()
    for w in words:
        x = c ^ (w & 0xFFFFFFFF)
        hi = w >> 32
        c = (t7[x & 0xFF] ^ t6[(x >> 8) & 0xFF] ^ t5[(x >> 16) & 0xFF] ^ t4[x >> 24] ^
             t3[hi & 0xFF] ^ t2[(hi >> 8) & 0xFF] ^ t1[(hi >> 16) & 0xFF] ^ t0[hi >> 24])
    for b in mv[n8:]:
        c = t0[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def mask_crc(crc: int) -> int:
    """LevelDB/TF masked CRC: rotate right by 15, add 0xa282ead8 (mod 2^32)."""
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(masked: int) -> int:
    rot = (masked - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------------
# varints and protobuf wire format
# ---------------------------------------------------------------------------
def _varint(buf, pos: int):
    result = shift = 0
    while True:
        if pos >= len(buf):
            raise ValueError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _proto_fields(buf):
    """Yield (field_number, wire_type, value) of a serialized protobuf message."""
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            if len(v) != ln:
                raise ValueError("truncated length-delimited field")
            pos += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield field, wt, v


def _parse_shape(buf):
    """TensorShapeProto: dim = 2 (TensorShapeProto.Dim: size = 1), unknown_rank = 3."""
    dims = []
    for f, wt, v in _proto_fields(buf):
        if f == 2 and wt == 2:
            size = 0
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    size = v2 - (1 << 64) if v2 >= 1 << 63 else v2
            dims.append(size)
        elif f == 3 and v:
            raise ValueError("tensor of unknown rank")
    return tuple(dims)


def parse_entry(buf) -> dict:
    """BundleEntryProto: dtype=1 shape=2 shard_id=3 offset=4 size=5 crc32c=6(fixed32) slices=7."""
    e = {"dtype": 0, "shape": (), "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": 0}
    for f, wt, v in _proto_fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2 and wt == 2:
            e["shape"] = _parse_shape(v)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = v
        elif f == 7:
            e["slices"] += 1
    return e


def parse_header(buf) -> dict:
    """BundleHeaderProto: num_shards=1 endianness=2 (0 little, 1 big) version=3 (VersionDef)."""
    h = {"num_shards": 1, "endianness": 0}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            h["num_shards"] = v
        elif f == 2:
            h["endianness"] = v
    return h


# ---------------------------------------------------------------------------
# sorted string table
# ---------------------------------------------------------------------------
def _read_block(data, offset: int, size: int, verify: bool):
    end = offset + size
    if end + BLOCK_TRAILER_LEN > len(data):
        raise ValueError("block handle past the end of the index file")
    block = data[offset:end]
    ctype = data[end]
    if verify:
        stored = struct.unpack_from("<I", data, end + 1)[0]
        if unmask_crc(stored) != crc32c(data[offset:end + 1]):
            raise ValueError(f"index block at {offset}: CRC-32C mismatch")
    if ctype != 0:
        raise ValueError(f"index block at {offset} is compressed (type {ctype}); only uncompressed tables are read")
    return block


def _block_entries(block):
    """Decode a table block: prefix-compressed (key, value) entries followed by the restart array."""
    if len(block) < 4:
        raise ValueError("block too short")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * nrest
    if limit < 0:
        raise ValueError("bad restart count")
    pos, key = 0, b""
    while pos < limit:
        shared, pos = _varint(block, pos)
        nonshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        if shared > len(key):
            raise ValueError("corrupt block entry")
        key = key[:shared] + bytes(block[pos:pos + nonshared])
        pos += nonshared
        yield key, bytes(block[pos:pos + vlen])
        pos += vlen


def read_table(data, verify: bool = True):
    """All (key, value) pairs of a LevelDB-format table (TF's tensorflow/core/lib/io/table)."""
    data = memoryview(data)
    if len(data) < FOOTER_LEN:
        raise ValueError("index file too short for a table footer")
    foot = data[len(data) - FOOTER_LEN:]
    if struct.unpack_from("<Q", foot, 40)[0] != TABLE_MAGIC:
        raise ValueError("not a TF tensor-bundle index (bad table magic)")
    pos = 0
    _, pos = _varint(foot, pos)          # metaindex offset
    _, pos = _varint(foot, pos)          # metaindex size
    ioff, pos = _varint(foot, pos)
    isize, pos = _varint(foot, pos)
    out = []
    for _, handle in _block_entries(_read_block(data, ioff, isize, verify)):
        boff, p = _varint(handle, 0)
        bsize, _ = _varint(handle, p)
        out.extend(_block_entries(_read_block(data, boff, bsize, verify)))
    return out


# ---------------------------------------------------------------------------
# the bundle
# ---------------------------------------------------------------------------
def _index_path(prefix: str) -> str:
    p = os.fspath(prefix)
    if p.endswith(".index"):
        p = p[:-len(".index")]
    return p


def list_variables(prefix):
    """[(name, shape)] of a checkpoint, like tf.train.list_variables."""
    p = _index_path(prefix)
    with open(p + ".index", "rb") as f:
        entries = read_table(f.read())
    return [(k.decode(), parse_entry(v)["shape"]) for k, v in entries if k]


def load_checkpoint(prefix, names=None, verify: bool = True) -> dict:
    """Read tensors of a TF1 (Saver V2) checkpoint prefix -> {name: np.ndarray}.

    ``names``: restrict to these tensor names (``:0`` suffixes are accepted and
    stripped).  Raises FileNotFoundError when ``<prefix>.index`` is missing (as TF's
    restore does), KeyError for a requested name that is absent, ValueError for a
    corrupt or unsupported file (compressed table, partitioned/sliced variable,
    bfloat16/string dtype, big-endian bundle, CRC mismatch).
    """
    p = _index_path(prefix)
    if not os.path.exists(p + ".index"):
        raise FileNotFoundError(f"checkpoint {p!r}: {p}.index not found")
    with open(p + ".index", "rb") as f:
        table = read_table(f.read(), verify)
    header = {"num_shards": 1, "endianness": 0}
    entries = {}
    for k, v in table:
        if not k:
            header = parse_header(v)
        else:
            entries[k.decode()] = v
    if header["endianness"] != 0:
        raise ValueError("big-endian tensor bundles are not supported")
    want = None if names is None else [n[:-2] if n.endswith(":0") else n for n in names]
    if want is not None:
        missing = [n for n in want if n not in entries]
        if missing:
            raise KeyError(f"checkpoint {p!r} lacks {missing}")
    out, files = {}, {}
    try:
        for name in (want if want is not None else sorted(entries)):
            e = parse_entry(entries[name])
            if e["slices"]:
                raise ValueError(f"{name}: partitioned (sliced) variables are not supported")
            if e["dtype"] not in _DTYPES:
                raise ValueError(f"{name}: unsupported dtype enum {e['dtype']}")
            dt = np.dtype(_DTYPES[e["dtype"]]).newbyteorder("<")
            n = int(np.prod(e["shape"], dtype=np.int64)) if e["shape"] else 1
            if e["size"] != n * dt.itemsize:
                raise ValueError(f"{name}: {e['size']} bytes for shape {e['shape']} of {dt}")
            shard = e["shard_id"]
            if shard not in files:
                path = f"{p}.data-{shard:05d}-of-{header['num_shards']:05d}"
                files[shard] = open(path, "rb")
            fh = files[shard]
            fh.seek(e["offset"])
            raw = fh.read(e["size"])
            if len(raw) != e["size"]:
                raise ValueError(f"{name}: data file truncated")
            if verify and e["crc32c"] is not None and unmask_crc(e["crc32c"]) != crc32c(raw):
                raise ValueError(f"{name}: tensor CRC-32C mismatch")
            out[name] = np.frombuffer(raw, dtype=dt).astype(dt.newbyteorder("="), copy=True).reshape(e["shape"])
    finally:
        for fh in files.values():
            fh.close()
    return out
