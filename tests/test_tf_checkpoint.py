"""TF1 tensor-bundle reader (scenedepthestimation_amd/tf_checkpoint.py) -- SURVEY.md sec. 8 row f4.

No TensorFlow and no checkpoint exist here (the reference's ./check_points_11_11 is not in
the repo), so parity with TF is unpinned; these tests pin the pieces that have published
answers (the CRC-32C check value and RFC 3720 vectors, the LevelDB mask) and round-trip
bundles written by the small writer below, which follows the published formats with
several data blocks, prefix-compressed keys and restart points like TF's TableBuilder.
"""
import struct

import numpy as np
import pytest

from scenedepthestimation_amd import mc_cnn, tf_checkpoint as tc


# ---------------------------------------------------------------- known answers
def test_crc32c_known_answers():
    assert tc.crc32c(b"123456789") == 0xE3069283             # the CRC-32C check value
    assert tc.crc32c(b"") == 0
    assert tc.crc32c(bytes(32)) == 0x8A9136AA                 # RFC 3720 B.4: 32 bytes of zeros
    assert tc.crc32c(b"\xff" * 32) == 0x62A8AB43              # ... 32 bytes of 0xff
    assert tc.crc32c(bytes(range(32))) == 0x46DD794E          # ... incrementing 0..31
    assert tc.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C  # ... decrementing 31..0
    # incremental use equals one pass
    assert tc.crc32c(b"6789", tc.crc32c(b"12345")) == 0xE3069283


def test_mask_roundtrip():
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF, 0x12345678):
        assert tc.unmask_crc(tc.mask_crc(c)) == c
    assert tc.mask_crc(0) == 0xA282EAD8


# ---------------------------------------------------------------- test writer
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_varint(f, v):
    return _varint(f << 3) + _varint(v)


def _field_bytes(f, b):
    return _varint((f << 3) | 2) + _varint(len(b)) + b


def _entry(dtype, shape, shard, offset, size, crc):
    shp = b"".join(_field_bytes(2, _field_varint(1, d)) for d in shape)
    return (_field_varint(1, dtype) + _field_bytes(2, shp) + _field_varint(3, shard) + _field_varint(4, offset) +
            _field_varint(5, size) + _varint((6 << 3) | 5) + struct.pack("<I", tc.mask_crc(crc)))


def _block(items, restart_interval):
    buf, restarts, prev = bytearray(), [], b""
    for i, (k, v) in enumerate(items):
        if i % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(prev)) and k[shared] == prev[shared]:
                shared += 1
        buf += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    for r in restarts or [0]:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts or [0]))
    return bytes(buf)


def _table(items, per_block=2, restart_interval=2, corrupt_block=None):
    out, index = bytearray(), []
    for bi in range(0, len(items), per_block):
        chunk = items[bi:bi + per_block]
        blk = _block(chunk, restart_interval)
        off = len(out)
        trailer = b"\x00" + struct.pack("<I", tc.mask_crc(tc.crc32c(blk + b"\x00")))
        if corrupt_block == bi // per_block:
            blk = bytes([blk[0] ^ 1]) + blk[1:]
        out += blk + trailer
        index.append((chunk[-1][0], _varint(off) + _varint(len(blk))))
    meta = _block([], 1)
    moff = len(out)
    out += meta + b"\x00" + struct.pack("<I", tc.mask_crc(tc.crc32c(meta + b"\x00")))
    iblk = _block(index, 1)
    ioff = len(out)
    out += iblk + b"\x00" + struct.pack("<I", tc.mask_crc(tc.crc32c(iblk + b"\x00")))
    foot = _varint(moff) + _varint(len(meta)) + _varint(ioff) + _varint(len(iblk))
    foot += bytes(40 - len(foot)) + struct.pack("<Q", tc.TABLE_MAGIC)
    return bytes(out + foot)


DT = {np.float32: 1, np.float64: 2, np.int32: 3, np.int64: 9}


def write_bundle(prefix, tensors, nshards=1, **kw):
    """Saver V2 layout: header under the empty key, entries sorted by name, data shards."""
    data = [bytearray() for _ in range(nshards)]
    items = [(b"", _field_varint(1, nshards))]
    for i, name in enumerate(sorted(tensors)):
        a = np.array(tensors[name], order="C")          # keeps 0-d shapes (ascontiguousarray does not)
        raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
        s = i % nshards
        items.append((name.encode(), _entry(DT[a.dtype.type], a.shape, s, len(data[s]), len(raw), tc.crc32c(raw))))
        data[s] += raw
    with open(str(prefix) + ".index", "wb") as f:
        f.write(_table(items, **kw))
    for s in range(nshards):
        with open(f"{prefix}.data-{s:05d}-of-{nshards:05d}", "wb") as f:
            f.write(bytes(data[s]))


# ---------------------------------------------------------------- round trips
def test_bundle_roundtrip_mc_cnn_names(tmp_path):
    w = mc_cnn.synthetic_weights(5, seed=7)
    tensors = {k[:-2]: v for k, v in w.items()}
    tensors["global_step"] = np.array(1400, np.int64)
    tensors["conv1/weights/Adam"] = np.ones((3, 3, 1, 64), np.float32)      # optimizer slots are ignored
    prefix = tmp_path / "model_epoch14.ckpt"
    write_bundle(prefix, tensors, nshards=2, per_block=3, restart_interval=2)
    names = dict(tc.list_variables(str(prefix)))
    assert names["conv3/weights"] == (3, 3, 64, 64) and names["global_step"] == ()
    got = mc_cnn.load_weights(str(prefix), 5)
    assert sorted(got) == sorted(w)
    for k in w:
        assert got[k].dtype == np.float32 and got[k].shape == w[k].shape
        assert got[k].tobytes() == w[k].tobytes()
    allt = tc.load_checkpoint(str(prefix) + ".index")
    assert int(allt["global_step"]) == 1400


def test_bundle_missing_and_corrupt(tmp_path):
    prefix = tmp_path / "m.ckpt"
    with pytest.raises(FileNotFoundError):
        tc.load_checkpoint(str(prefix))
    write_bundle(prefix, {"conv1/weights": np.zeros((3, 3, 1, 64), np.float32)})
    with pytest.raises(KeyError):
        mc_cnn.load_weights(str(prefix), 5)                 # conv1/biases ... absent
    # flipped tensor byte -> CRC mismatch
    dpath = f"{prefix}.data-00000-of-00001"
    raw = bytearray(open(dpath, "rb").read())
    raw[5] ^= 0x40
    open(dpath, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="CRC"):
        tc.load_checkpoint(str(prefix))
    # corrupt index block
    p2 = tmp_path / "n.ckpt"
    write_bundle(p2, {"a": np.arange(6, dtype=np.float32), "b": np.arange(3, dtype=np.int32)}, corrupt_block=0)
    with pytest.raises(ValueError, match="CRC"):
        tc.load_checkpoint(str(p2))
    # not a table
    p3 = tmp_path / "o.ckpt"
    open(str(p3) + ".index", "wb").write(bytes(64))
    with pytest.raises(ValueError, match="magic"):
        tc.load_checkpoint(str(p3))
