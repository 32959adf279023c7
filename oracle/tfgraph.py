"""ORACLE (test infrastructure only) -- a reader for the reference's TensorBoard event files
and a small numpy interpreter for the TensorFlow-1 GraphDefs they carry.

The reference ships the graphs its drivers built, as TensorBoard logs:
    src/~/reacher/data/viz/1/events.out.tfevents.*     (12 files, TF 1.10)
Each file is a TFRecord stream (u64 length, u32 masked crc, payload, u32 masked crc) of
`Event` protos; one of them holds `graph_def` (Event field 4): the NodeDefs of the teacher's
baselines MlpPolicy (`pi/...`), an LSTM student variant (`LSTM/...`, TF1 LSTMCell
`unique_lstm_cell`, the kl loss of reference loss.py:3-13), the TF-generated backward
(`adam/gradients/...`) and the Adam update (`adam/Adam/...`, ApplyAdam).

These files are DATA: they are parsed with a protobuf wire-format reader written here
(no TensorFlow, nothing in them is executed as code).  `Graph.run` evaluates a subgraph in
float64 with numpy so that the reference's own computation (ops, wiring, constants) can be
compared against this repo's oracles (`tests/golden/make_graph_consts.py` writes the
results as golden vectors; `tests/test_graph_pins.py` checks the oracles against them).

Interpreted op set (the subset these graphs use): Const, Placeholder/VariableV2 (fed),
Identity, Cast, Sub, Add, AddN, Mul, RealDiv, Neg, Square, Sqrt, Exp, Tanh, Sigmoid, Floor,
Maximum, Minimum, MatMul, BiasAdd, BiasAddGrad, TanhGrad, SigmoidGrad, ConcatV2,
ConcatOffset, Split, Pack, Unpack, StridedSlice (begin/end/shrink masks), Slice, Squeeze,
Sum, Reshape, Shape, Fill, Tile, BroadcastGradientArgs, Range, FloorMod, FloorDiv,
DynamicStitch.
"""
from __future__ import annotations

import glob
import os
import struct

import numpy as np

REF_VIZ = "/root/reference/src/~/reacher/data/viz/1"

# TF DataType enum -> numpy (types.proto)
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_}


# ------------------------------------------------------------------ protobuf wire format
def _varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _fields(b):
    """(field number, wire type, value) of one message; value = int | bytes."""
    i = 0
    while i < len(b):
        k, i = _varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 2:
            n, i = _varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def _signed(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def _packed_varints(v):
    out, j = [], 0
    while j < len(v):
        x, j = _varint(v, j)
        out.append(_signed(x))
    return out


def records(path):
    """Payloads of a TFRecord file (lengths checked, crcs skipped)."""
    with open(path, "rb") as fh:
        d = fh.read()
    i = 0
    while i < len(d):
        n = struct.unpack_from("<Q", d, i)[0]
        i += 12
        if i + n + 4 > len(d):
            raise ValueError(f"{path}: truncated record")
        yield d[i:i + n]
        i += n + 4


def _shape(b):   # TensorShapeProto: dim (2) { size (1) }
    return [dict((f, v) for f, _, v in _fields(d)).get(1, 0) for f, _, d in _fields(b) if f == 2]


def _tensor(b):
    """TensorProto -> numpy array (dtype 1, shape 2, tensor_content 4, float_val 5,
    double_val 6, int_val 7, int64_val 10, bool_val 11)."""
    dt, shp, content, vals = 1, [], None, []
    for f, w, v in _fields(b):
        if f == 1:
            dt = v
        elif f == 2:
            shp = _shape(v)
        elif f == 4:
            content = v
        elif f == 5:
            vals += list(np.frombuffer(v, "<f4")) if w == 2 else [struct.unpack("<f", v)[0]]
        elif f == 6:
            vals += list(np.frombuffer(v, "<f8")) if w == 2 else [struct.unpack("<d", v)[0]]
        elif f in (7, 10):
            vals += _packed_varints(v) if w == 2 else [_signed(v)]
        elif f == 11:
            vals += [bool(x) for x in _packed_varints(v)] if w == 2 else [bool(v)]
    t = _DT.get(dt)
    if t is None:
        return None
    n = int(np.prod(shp)) if shp else 1
    if content is not None:
        a = np.frombuffer(content, np.dtype(t).newbyteorder("<")).astype(t)
    else:
        a = np.array(vals, t)
        if a.size == 1 and n > 1:   # a splat constant
            a = np.full(n, a[0], t)
    return a.reshape(shp)


def _attr(b):
    """AttrValue -> python: s (2) str, i (3) int, f (4) float, b (5) bool, type (6),
    shape (7), tensor (8), list (1: its i / type / shape entries)."""
    for f, w, v in _fields(b):
        if f == 2:
            return v.decode(errors="replace")
        if f == 3:
            return _signed(v)
        if f == 4:
            return struct.unpack("<f", v)[0]
        if f == 5:
            return bool(v)
        if f == 6:
            return ("type", v)
        if f == 7:
            return ("shape", _shape(v))
        if f == 8:
            return _tensor(v)
        if f == 1:
            ints = []
            for ff, ww, vv in _fields(v):
                if ff == 3:
                    ints += _packed_varints(vv) if ww == 2 else [_signed(vv)]
            return ("list", ints)
    return None


def graph_defs(path):
    """The GraphDefs of one event file, as {name: node dict}."""
    out = []
    for rec in records(path):
        for f, _, v in _fields(rec):
            if f != 4:       # Event.graph_def
                continue
            nodes = {}
            for ff, _, nv in _fields(v):
                if ff != 1:  # GraphDef.node
                    continue
                nd = dict(name="", op="", inputs=[], attr={})
                for a, _, x in _fields(nv):
                    if a == 1:
                        nd["name"] = x.decode()
                    elif a == 2:
                        nd["op"] = x.decode()
                    elif a == 3:
                        nd["inputs"].append(x.decode())
                    elif a == 5:   # map<string, AttrValue> entry
                        kv = dict((k, y) for k, _, y in _fields(x))
                        nd["attr"][kv[1].decode()] = _attr(kv.get(2, b""))
                nodes[nd["name"]] = nd
            out.append(nodes)
    return out


def event_files(root=REF_VIZ):
    return sorted(glob.glob(os.path.join(root, "events.out.tfevents.*")))


# ------------------------------------------------------------------ interpreter
class Graph:
    """Evaluate nodes of a GraphDef in float64 (integer tensors stay integer)."""

    def __init__(self, nodes):
        self.nodes = nodes

    def const(self, name):
        nd = self.nodes[name]
        assert nd["op"] == "Const", (name, nd["op"])
        return nd["attr"]["value"]

    def run(self, fetches, feeds):
        cache = {}
        for k, v in feeds.items():   # float feeds are evaluated in float64 like the constants
            cache[k if ":" in k else k + ":0"] = self._f(v)
        single = isinstance(fetches, str)
        out = [self._value(f, cache) for f in ([fetches] if single else fetches)]
        return out[0] if single else out

    def _value(self, ref, cache):
        name, idx = (ref.rsplit(":", 1) if ":" in ref else (ref, "0"))
        key = f"{name}:{idx}"
        if key in cache:
            return cache[key]
        if name not in self.nodes:
            raise KeyError(f"no node {name}")
        nd = self.nodes[name]
        ins = [self._value(i, cache) for i in nd["inputs"] if not i.startswith("^")]
        outs = self._eval(nd, ins)
        if not isinstance(outs, list):
            outs = [outs]
        for k, o in enumerate(outs):
            cache[f"{name}:{k}"] = o
        return cache[key]

    @staticmethod
    def _f(x):
        x = np.asarray(x)
        return x.astype(np.float64) if x.dtype.kind == "f" else x

    def _eval(self, nd, x):  # noqa: C901  (one branch per op)
        op, at = nd["op"], nd["attr"]
        f = self._f
        if op == "Const":
            return f(at["value"])
        if op in ("Placeholder", "VariableV2"):
            raise KeyError(f"{nd['name']} ({op}) must be fed")
        if op in ("Identity", "Snapshot", "StopGradient"):
            return x[0]
        if op == "Cast":   # float widths collapse to f64 here; integer casts are real
            dst = _DT[at["DstT"][1]]
            return f(x[0]) if np.dtype(dst).kind == "f" else np.asarray(x[0]).astype(dst)
        binop = {"Sub": np.subtract, "Add": np.add, "Mul": np.multiply, "RealDiv": np.divide,
                 "Maximum": np.maximum, "Minimum": np.minimum, "FloorMod": np.mod,
                 "FloorDiv": np.floor_divide}
        if op in binop:
            return binop[op](x[0], x[1])
        unop = {"Neg": np.negative, "Square": np.square, "Sqrt": np.sqrt, "Exp": np.exp,
                "Tanh": np.tanh, "Floor": np.floor, "Sigmoid": lambda v: 1.0 / (1.0 + np.exp(-v))}
        if op in unop:
            return unop[op](f(x[0]))
        if op == "AddN":
            s = x[0]
            for v in x[1:]:
                s = s + v
            return s
        if op == "TanhGrad":      # (y, dy) -> dy (1 - y^2)
            return x[1] * (1.0 - x[0] * x[0])
        if op == "SigmoidGrad":   # (y, dy) -> dy y (1 - y)
            return x[1] * x[0] * (1.0 - x[0])
        if op == "MatMul":
            a = x[0].T if at.get("transpose_a") else x[0]
            b = x[1].T if at.get("transpose_b") else x[1]
            return a @ b
        if op == "BiasAdd":
            return x[0] + x[1]
        if op == "BiasAddGrad":
            return x[0].reshape(-1, x[0].shape[-1]).sum(0)
        if op == "ConcatV2":
            ax = int(x[-1])
            return np.concatenate(x[:-1], axis=ax)
        if op == "ConcatOffset":   # (axis, shapes...) -> offsets of each input along axis
            ax, shapes = int(x[0]), x[1:]
            offs, o = [], 0
            for s in shapes:
                v = np.zeros_like(s)
                v[ax] = o
                offs.append(v)
                o += int(s[ax])
            return offs
        if op == "Split":
            return list(np.split(x[1], at["num_split"], axis=int(x[0])))
        if op == "Pack":
            return np.stack(x, axis=at.get("axis", 0))
        if op == "Unpack":
            ax = at.get("axis", 0)
            return [np.take(x[0], k, axis=ax) for k in range(x[0].shape[ax])]
        if op == "StridedSlice":
            return self._strided_slice(x, at)
        if op == "Slice":
            beg, size = x[1], x[2]
            sl = tuple(slice(int(b), None if int(s) < 0 else int(b) + int(s)) for b, s in zip(beg, size))
            return x[0][sl]
        if op == "Squeeze":
            dims = at.get("squeeze_dims", ("list", []))[1]
            return np.squeeze(x[0], axis=tuple(dims)) if dims else np.squeeze(x[0])
        if op == "Sum":
            ax = tuple(int(a) for a in np.atleast_1d(x[1]))
            return np.sum(x[0], axis=ax, keepdims=bool(at.get("keep_dims", False)))
        if op == "Reshape":
            return np.reshape(x[0], [int(v) for v in np.atleast_1d(x[1])])
        if op == "Shape":
            return np.array(np.shape(x[0]), np.int32)
        if op == "Fill":
            return np.full([int(v) for v in np.atleast_1d(x[0])], x[1])
        if op == "Tile":
            return np.tile(x[0], [int(v) for v in x[1]])
        if op == "Range":
            return np.arange(int(x[0]), int(x[1]), int(x[2]), dtype=np.int32)
        if op == "BroadcastGradientArgs":
            return self._bcast_args(x[0], x[1])
        if op == "DynamicStitch":
            n = len(x) // 2
            idx, dat = x[:n], x[n:]
            size = max(int(np.max(i)) for i in idx) + 1
            out = np.zeros(size, dtype=np.asarray(dat[0]).dtype)
            for i, d in zip(idx, dat):
                out[np.asarray(i).ravel()] = np.asarray(d).ravel()
            return out
        raise NotImplementedError(f"op {op} ({nd['name']})")

    @staticmethod
    def _strided_slice(x, at):
        v, beg, end, st = x[0], x[1], x[2], x[3]
        bm, em, sm = at.get("begin_mask", 0), at.get("end_mask", 0), at.get("shrink_axis_mask", 0)
        if at.get("ellipsis_mask", 0) or at.get("new_axis_mask", 0):
            raise NotImplementedError("StridedSlice ellipsis/new-axis masks")
        sl = []
        for d in range(len(beg)):
            if sm >> d & 1:
                sl.append(int(beg[d]))
                continue
            b = None if bm >> d & 1 else int(beg[d])
            e = None if em >> d & 1 else int(end[d])
            sl.append(slice(b, e, int(st[d])))
        return v[tuple(sl)]

    @staticmethod
    def _bcast_args(s0, s1):
        """Reduction indices for the gradients of a broadcasting binary op."""
        s0, s1 = [int(v) for v in s0], [int(v) for v in s1]
        n = max(len(s0), len(s1))
        a = [1] * (n - len(s0)) + s0
        b = [1] * (n - len(s1)) + s1
        r0 = [i for i in range(n) if a[i] == 1 and b[i] != 1]
        r1 = [i for i in range(n) if b[i] == 1 and a[i] != 1]
        return [np.array(r0, np.int32), np.array(r1, np.int32)]


def reference_graph(root=REF_VIZ):
    """The first GraphDef of the reference's event files (all 12 share the teacher and
    the optimiser constants; tests/golden/make_graph_consts.py checks that)."""
    for p in event_files(root):
        gds = graph_defs(p)
        if gds:
            return Graph(gds[0]), p
    raise FileNotFoundError(f"no GraphDef under {root}")
