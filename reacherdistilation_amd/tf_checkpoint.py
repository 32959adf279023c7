"""TensorFlow-1 checkpoints (the V2 tensor bundle that ``tf.train.Saver`` writes) without
TensorFlow: read, write, and the teacher's variable mapping.

The reference restores its teacher with ``tf.train.Saver(var_list=<GLOBAL_VARIABLES in scope
'pi'>).restore(sess, "<base>/teacher.ckpt")`` (reference teacher.py:17-20) and saves / restores
the LSTM student the same way (lstm_train.py:86-107,199).  No checkpoint ships with the
reference, so this module follows TensorFlow's published on-disk format (tensor_bundle.proto and
the LevelDB-style table of core/lib/io/table_builder.cc, TF 1.10):

``<prefix>.index``  an SSTable: data blocks of prefix-compressed (key, value) entries with restart
                    points, a metaindex block (empty), an index block (separator key -> block
                    handle), each block followed by a 5-byte trailer (compression type 0 + masked
                    CRC32C), and a 48-byte footer (two block handles, padding, magic
                    0xdb4775248b80fb57).  Key "" holds a BundleHeaderProto, every other key (the
                    variable name) a BundleEntryProto {dtype, shape, shard_id, offset, size,
                    crc32c (masked)}.
``<prefix>.data-00000-of-00001``  the tensors' raw little-endian bytes, back to back.

The variable list of the teacher (names, order, dtypes, shapes) is pinned to the Saver node
``save/SaveV2`` of the reference's own logged GraphDef (tests/test_tf_checkpoint.py), and the
observation filter's restore arithmetic to that graph's ``pi/obfilter`` ops.  The byte format is
checked by round trips and the published CRC32C check value; no TensorFlow-written file is
available to pin it ("parity unpinned" for the bytes).
"""
from __future__ import annotations

import os
import struct

import numpy as np

from .policy import ACD, HID, OBD, P_TOT, SLICES, MlpPolicyParams

# ------------------------------------------------------------------ CRC32C (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)
_TABLE = np.array(_TABLE, np.uint32)


def crc32c_py(data: bytes, crc: int = 0) -> int:
    """The per-byte table form (the definition the native one is tested against)."""
    c = crc ^ 0xFFFFFFFF
    t = _TABLE
    for b in data:
        c = int(t[(c ^ b) & 0xFF]) ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def crc32c(data: bytes, crc: int = 0) -> int:
    """CRC32C of `data`, continuing from `crc`: the native form (rd_crc32c in libreacher.so:
    the SSE4.2 crc32 instruction, else slicing-by-8), else crc32c_py (~2 MB/s)."""
    try:
        from . import _native
        lib = _native.load()
    except Exception:   # noqa: BLE001  (host utility: the library is the fast path, not a requirement)
        return crc32c_py(data, crc)
    import ctypes
    b = data if isinstance(data, bytes) else bytes(data)
    buf = ctypes.c_char_p(b) if b else None   # points into the bytes object: no copy
    return int(lib.rd_crc32c(buf, len(b), crc & 0xFFFFFFFF))


def _mask(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _unmask(m: int) -> int:
    r = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------ protobuf wire format
def _uvarint(x: int) -> bytes:
    out = bytearray()
    x &= (1 << 64) - 1
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_uvarint(b: bytes, i: int):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_uvarint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_uvarint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 2:
            n, i = _read_uvarint(b, i)
            v, i = b[i:i + n], i + n
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def _key(f: int, w: int) -> bytes:
    return _uvarint((f << 3) | w)


def _len_field(f: int, payload: bytes) -> bytes:
    return _key(f, 2) + _uvarint(len(payload)) + payload


# TF DataType enum (types.proto) <-> numpy
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_, 19: np.float16}
_DT_OF = {np.dtype(v): k for k, v in _DT.items()}


def _shape_proto(shape) -> bytes:
    return b"".join(_len_field(2, _key(1, 0) + _uvarint(int(d))) for d in shape)


def _parse_shape(b: bytes):
    dims = []
    for f, _, v in _fields(b):
        if f == 2:
            size = 0
            for ff, _, vv in _fields(v):
                if ff == 1:
                    size = vv - (1 << 64) if vv >= 1 << 63 else vv
            dims.append(size)
    return tuple(dims)


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    out = _key(1, 0) + _uvarint(dtype) + _len_field(2, _shape_proto(shape))
    # shard_id 0 is the default (omitted, as proto3 serialisation does)
    if offset:
        out += _key(4, 0) + _uvarint(offset)
    if size:
        out += _key(5, 0) + _uvarint(size)
    return out + _key(6, 5) + struct.pack("<I", crc)


def _parse_entry(b: bytes) -> dict:
    e = dict(dtype=0, shape=(), shard_id=0, offset=0, size=0, crc32c=None, slices=False)
    for f, _, v in _fields(b):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            e["shape"] = _parse_shape(v)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = struct.unpack("<I", v)[0]
        elif f == 7:
            e["slices"] = True
    return e


def _header_proto(num_shards: int = 1) -> bytes:
    # num_shards (1), endianness (2) = LITTLE (0, omitted), version (3) = VersionDef{producer 1}
    return _key(1, 0) + _uvarint(num_shards) + _len_field(3, _key(1, 0) + _uvarint(1))


def _parse_header(b: bytes) -> dict:
    h = dict(num_shards=1, endianness=0, producer=0)
    for f, _, v in _fields(b):
        if f == 1:
            h["num_shards"] = v
        elif f == 2:
            h["endianness"] = v
        elif f == 3:
            for ff, _, vv in _fields(v):
                if ff == 1:
                    h["producer"] = vv
    return h


# ------------------------------------------------------------------ SSTable (table format)
_MAGIC = 0xDB4775248B80FB57
_FOOTER = 48


def _block(entries, restart_interval: int) -> bytes:
    """One table block: prefix-compressed entries, restart offsets, restart count."""
    out = bytearray()
    restarts, prev = [], b""
    for n, (k, v) in enumerate(entries):
        if n % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _uvarint(shared) + _uvarint(len(k) - shared) + _uvarint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _block_entries(blk: bytes):
    nres = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    end = len(blk) - 4 - 4 * nres
    i, key = 0, b""
    while i < end:
        shared, i = _read_uvarint(blk, i)
        non, i = _read_uvarint(blk, i)
        vlen, i = _read_uvarint(blk, i)
        key = key[:shared] + blk[i:i + non]
        i += non
        yield key, blk[i:i + vlen]
        i += vlen


def _handle(offset: int, size: int) -> bytes:
    return _uvarint(offset) + _uvarint(size)


def _read_block(buf: bytes, offset: int, size: int) -> bytes:
    blk = buf[offset:offset + size]
    typ = buf[offset + size]
    crc = struct.unpack_from("<I", buf, offset + size + 1)[0]
    if typ != 0:
        raise ValueError("compressed table blocks are not supported (TF writes bundles uncompressed)")
    if _unmask(crc) != crc32c(blk + bytes([typ])):
        raise ValueError("table block checksum mismatch")
    return blk


def _table(entries) -> bytes:
    """An SSTable of sorted (key, value) byte pairs: one data block per 4 KiB, restart interval
    16 (index block: 1), no compression, as TF's table builder writes a bundle index."""
    out = bytearray()
    index = []

    def emit(blk):
        off = len(out)
        out.extend(blk)
        out.append(0)
        out.extend(struct.pack("<I", _mask(crc32c(blk + b"\x00"))))
        return off, len(blk)

    cur, size = [], 0
    for k, v in entries:
        cur.append((k, v))
        size += len(k) + len(v) + 8
        if size >= 4096:
            index.append((cur[-1][0], emit(_block(cur, 16))))
            cur, size = [], 0
    if cur:
        index.append((cur[-1][0], emit(_block(cur, 16))))
    meta = emit(_block([], 16))
    idx = emit(_block([(k, _handle(*h)) for k, h in index], 1))
    footer = _handle(*meta) + _handle(*idx)
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<II", _MAGIC & 0xFFFFFFFF, _MAGIC >> 32)
    return bytes(out) + footer


def _read_table(buf: bytes):
    if len(buf) < _FOOTER:
        raise ValueError("not a table: shorter than its footer")
    lo, hi = struct.unpack_from("<II", buf, len(buf) - 8)
    if (hi << 32 | lo) != _MAGIC:
        raise ValueError("not a TensorFlow checkpoint index (bad table magic)")
    f = buf[len(buf) - _FOOTER:len(buf) - 8]
    _, i = _read_uvarint(f, 0)      # metaindex handle (unused)
    _, i = _read_uvarint(f, i)
    io, i = _read_uvarint(f, i)
    isz, i = _read_uvarint(f, i)
    for _, h in _block_entries(_read_block(buf, io, isz)):
        off, j = _read_uvarint(h, 0)
        size, _ = _read_uvarint(h, j)
        yield from _block_entries(_read_block(buf, off, size))


# ------------------------------------------------------------------ bundle read / write
def _data_path(prefix: str, shard: int, num_shards: int) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def read(prefix: str) -> dict:
    """{variable name: numpy array} of the checkpoint ``prefix`` (``prefix.index`` + data
    shards).  Raises ValueError on a checksum mismatch, a big-endian or sliced bundle, or a
    dtype other than float16/32/64, int32/64, bool."""
    with open(prefix + ".index", "rb") as fh:
        buf = fh.read()
    header, entries = None, {}
    for k, v in _read_table(buf):
        if k == b"":
            header = _parse_header(v)
        else:
            entries[k.decode()] = _parse_entry(v)
    if header is None:
        raise ValueError("checkpoint index without a bundle header")
    if header["endianness"] != 0:
        raise ValueError("big-endian bundles are not supported")
    shards = {}
    out = {}
    for name, e in entries.items():
        if e["slices"]:
            raise ValueError(f"{name}: partitioned (sliced) variables are not supported")
        dt = _DT.get(e["dtype"])
        if dt is None:
            raise ValueError(f"{name}: unsupported dtype enum {e['dtype']}")
        sid = e["shard_id"]
        if sid not in shards:
            with open(_data_path(prefix, sid, header["num_shards"]), "rb") as fh:
                shards[sid] = fh.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(raw) != e["size"]:
            raise ValueError(f"{name}: data shard too short")
        if e["crc32c"] is not None and _unmask(e["crc32c"]) != crc32c(raw):
            raise ValueError(f"{name}: tensor checksum mismatch")
        a = np.frombuffer(raw, np.dtype(dt).newbyteorder("<")).astype(dt)
        out[name] = a.reshape(e["shape"])
    return out


def write(prefix: str, tensors: dict) -> None:
    """Write ``tensors`` ({name: array}) as a single-shard V2 bundle at ``prefix``, keys in
    byte order as TF's BundleWriter emits them."""
    d = os.path.dirname(os.path.abspath(prefix))
    os.makedirs(d, exist_ok=True)
    data = bytearray()
    rows = [(b"", _header_proto(1))]
    for name in sorted(tensors, key=lambda s: s.encode()):
        a = np.asarray(tensors[name])
        a = a if a.flags.c_contiguous else a.copy(order="C")   # (ascontiguousarray makes 0-d 1-d)
        if a.dtype not in _DT_OF:
            raise ValueError(f"{name}: unsupported dtype {a.dtype}")
        raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
        rows.append((name.encode(), _entry_proto(_DT_OF[a.dtype], a.shape, len(data), len(raw),
                                                 _mask(crc32c(raw)))))
        data += raw
    with open(_data_path(prefix, 0, 1), "wb") as fh:
        fh.write(bytes(data))
    with open(prefix + ".index", "wb") as fh:
        fh.write(_table(rows))


def exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".index")


# ------------------------------------------------------------------ the teacher (scope 'pi')
# The reference teacher Saver's variables in its SaveV2 input order (baselines ppo1 MlpPolicy,
# hid_size 64, num_hid_layers 2, reference teacher.py:14-18): name, shape, dtype
TEACHER_VARS = [
    ("pi/obfilter/runningsum", (OBD,), np.float64),
    ("pi/obfilter/runningsumsq", (OBD,), np.float64),
    ("pi/obfilter/count", (), np.float64),
    ("pi/vf/fc1/kernel", (OBD, HID), np.float32), ("pi/vf/fc1/bias", (HID,), np.float32),
    ("pi/vf/fc2/kernel", (HID, HID), np.float32), ("pi/vf/fc2/bias", (HID,), np.float32),
    ("pi/vf/final/kernel", (HID, 1), np.float32), ("pi/vf/final/bias", (1,), np.float32),
    ("pi/pol/fc1/kernel", (OBD, HID), np.float32), ("pi/pol/fc1/bias", (HID,), np.float32),
    ("pi/pol/fc2/kernel", (HID, HID), np.float32), ("pi/pol/fc2/bias", (HID,), np.float32),
    ("pi/pol/final/kernel", (HID, ACD), np.float32), ("pi/pol/final/bias", (ACD,), np.float32),
    ("pi/pol/logstd", (1, ACD), np.float32),
]
_POL = [("W1", "pi/pol/fc1/kernel"), ("b1", "pi/pol/fc1/bias"), ("W2", "pi/pol/fc2/kernel"),
        ("b2", "pi/pol/fc2/bias"), ("W3", "pi/pol/final/kernel"), ("b3", "pi/pol/final/bias"),
        ("logstd", "pi/pol/logstd")]


def obfilter(runningsum, runningsumsq, count):
    """baselines RunningMeanStd as the graph computes it (the reference GraphDef's pi/obfilter
    ops): mean = f32(sum / count), std = sqrt(max(f32(sumsq / count) - mean^2, 1e-2))."""
    s, q, c = (np.asarray(x, np.float64) for x in (runningsum, runningsumsq, count))
    mean = (s / c).astype(np.float32)
    var = (q / c).astype(np.float32) - np.square(mean)
    return mean, np.sqrt(np.maximum(var, np.float32(1e-2))).astype(np.float32)


def load_teacher(prefix: str) -> MlpPolicyParams:
    """The teacher's MlpPolicy (policy head + observation filter) from a checkpoint written by
    the reference's Saver (teacher.py:17-20) or by ``save_teacher``; the value head is unused."""
    t = read(prefix)
    missing = [n for n, _, _ in TEACHER_VARS if n not in t]
    if missing:
        raise KeyError(f"{prefix}: not a scope-'pi' MlpPolicy checkpoint, missing {missing}")
    for n, shape, dt in TEACHER_VARS:
        if tuple(t[n].shape) != shape:
            raise ValueError(f"{n}: shape {t[n].shape}, expected {shape}")
    flat = np.zeros(P_TOT, np.float32)
    for key, name in _POL:
        a, b, _ = SLICES[key]
        flat[a:b] = t[name].astype(np.float32).ravel()
    mean, std = obfilter(t["pi/obfilter/runningsum"], t["pi/obfilter/runningsumsq"], t["pi/obfilter/count"])
    return MlpPolicyParams(flat, mean, std)


def save_teacher(prefix: str, p: MlpPolicyParams, vf: dict | None = None, count: float = 1e4) -> None:
    """Write ``p`` as the reference Saver's scope-'pi' checkpoint (every variable it restores):
    the filter as running sums over ``count`` samples that reproduce p.ob_mean / p.ob_std
    (std >= 0.1, the filter's floor), the value head from ``vf`` ({name: array}) or zeros."""
    mean = np.asarray(p.ob_mean, np.float64)
    std = np.asarray(p.ob_std, np.float64)
    if np.any(std < 0.1 - 1e-7):
        raise ValueError("ob_std below the RunningMeanStd floor sqrt(1e-2) cannot be represented")
    c = np.float64(count)
    out = {"pi/obfilter/runningsum": mean * c, "pi/obfilter/runningsumsq": (std * std + mean * mean) * c,
           "pi/obfilter/count": np.array(c, np.float64)}
    for n, shape, dt in TEACHER_VARS[3:9]:
        out[n] = np.asarray((vf or {}).get(n, np.zeros(shape)), dt).reshape(shape)
    for key, name in _POL:
        shape = dict((n, s) for n, s, _ in TEACHER_VARS)[name]
        out[name] = np.asarray(p[key], np.float32).reshape(shape)
    write(prefix, out)


# ------------------------------------------------------------------ the LSTM student (scope 'LSTM')
# lstm_train.py:86-87 saves / restores tf.train.Saver(var_list=<GLOBAL_VARIABLES in scope 'LSTM'>):
# the student's variables and their Adam slots ('<var>/Adam' = m, '<var>/Adam_1' = v; the beta
# powers live in scope 'adam' and are not saved).  Variable names follow TF1's layer naming in
# student_lstm_graph (student_nn.py:21-49): the prev-pdflat dense is the scope's first
# tf.layers.dense ('dense'), the cell 'unique_lstm_cell', and step t's five head layers the
# un-reused calls 5t+1 .. 5t+5 ('dense_1' ..).  The cell's name matches the reference's logged
# GraphDef (LSTM/unique_lstm_cell/kernel); the dense names follow TF1's uniquing rule (the
# logged graph is an older variant with named per-step layers), so they are unpinned.
def lstm_variables(T: int):
    """[(checkpoint name, flat offset, shape)] of the student in its flat order
    (student_lstm.shapes)."""
    from .student_lstm import CELL_SHAPES, HEAD_SHAPES, shapes
    names = {"Wp": "LSTM/dense/kernel", "bp": "LSTM/dense/bias", "Wl": "LSTM/unique_lstm_cell/kernel",
             "bl": "LSTM/unique_lstm_cell/bias"}
    out, off = [], 0
    for key, shp in shapes(T):
        if "/" in key:   # h{t}/W{k} or h{t}/b{k}
            t, layer = key.split("/")
            k = int(layer[1:])
            name = f"LSTM/dense_{5 * int(t[1:]) + k}/{'kernel' if layer[0] == 'W' else 'bias'}"
        else:
            name = names[key]
        out.append((name, off, tuple(shp)))
        off += int(np.prod(shp))
    assert len(out) == len(CELL_SHAPES) + len(HEAD_SHAPES) * T
    return out


def save_lstm(prefix: str, params, m=None, v=None, T: int = 10) -> None:
    """The flat parameters (and Adam slots m, v) as the reference's 'LSTM'-scope checkpoint."""
    params = np.asarray(params, np.float32).ravel()
    out = {}
    for name, off, shp in lstm_variables(T):
        n = int(np.prod(shp))
        out[name] = params[off:off + n].reshape(shp)
        for suffix, slot in (("/Adam", m), ("/Adam_1", v)):
            if slot is not None:
                out[name + suffix] = np.asarray(slot, np.float32).ravel()[off:off + n].reshape(shp)
    write(prefix, out)


def load_lstm(prefix: str, T: int = 10):
    """(params, m, v) flat float32 arrays from an 'LSTM'-scope checkpoint (m / v None when the
    checkpoint holds no Adam slots)."""
    t = read(prefix)
    var = lstm_variables(T)
    n = var[-1][1] + int(np.prod(var[-1][2]))
    missing = [name for name, _, _ in var if name not in t]
    if missing:
        raise KeyError(f"{prefix}: not a T = {T} LSTM-student checkpoint, missing {missing[:4]}"
                       f"{' ...' if len(missing) > 4 else ''}")
    out = []
    for suffix in ("", "/Adam", "/Adam_1"):
        if suffix and any(name + suffix not in t for name, _, _ in var):
            out.append(None)
            continue
        flat = np.zeros(n, np.float32)
        for name, off, shp in var:
            a = t[name + suffix]
            if tuple(a.shape) != shp:
                raise ValueError(f"{name + suffix}: shape {a.shape}, expected {shp}")
            flat[off:off + a.size] = a.astype(np.float32).ravel()
        out.append(flat)
    return tuple(out)
