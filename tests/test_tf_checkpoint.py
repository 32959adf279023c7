"""TF1 V2-bundle checkpoints without TensorFlow (reacherdistilation_amd/tf_checkpoint.py): the
reference restores its teacher with tf.train.Saver (reference teacher.py:17-20).  No checkpoint
file ships with the reference, so the BYTE format is checked against TensorFlow's published
format only (round trips, the table/footer/CRC invariants, the CRC32C check value: parity
unpinned); the teacher's VARIABLES -- names, shapes, dtypes, the Saver's key set -- and the
observation filter's restore arithmetic are pinned to the reference's own logged GraphDef
(its save/SaveV2 node and pi/obfilter ops)."""
import os
import struct

import numpy as np
import pytest

from reacherdistilation_amd import tf_checkpoint as tc
from reacherdistilation_amd.policy import MlpPolicyParams, TeacherAgent, synthetic_teacher


def test_crc32c_check_value():
    assert tc.crc32c(b"123456789") == 0xE3069283          # the CRC-32C (Castagnoli) check value
    assert tc.crc32c(b"") == 0
    for v in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert tc._unmask(tc._mask(v)) == v


def test_native_crc32c_matches_the_table_definition():
    """rd_crc32c (libreacher.so: SSE4.2 crc32 where the CPU has it) = the per-byte table form on
    every length 0..70 (all tail cases of the 8-byte loop), on a 1 MB buffer, and when continued
    in pieces."""
    rs = np.random.RandomState(0)
    data = rs.randint(0, 256, 1 << 20).astype(np.uint8).tobytes()
    for n in range(71):
        assert tc.crc32c(data[:n]) == tc.crc32c_py(data[:n]), n
    big = tc.crc32c(data)
    assert big == tc.crc32c_py(data)
    assert tc.crc32c(data[600_001:], tc.crc32c(data[:600_001])) == big


def test_native_crc32c_table_form_matches(tmp_path):
    """The slicing-by-8 form (what a CPU without SSE4.2 runs) gives the same CRCs: the same source
    built on the host with the CPU probe answering "no", called on every tail length and a
    200 KB buffer, continued in pieces."""
    import ctypes
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not found")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = str(tmp_path / "libcrc_tables.so")
    src = tmp_path / "crc_tables.cpp"
    src.write_text('#define __builtin_cpu_supports(feature) 0\n#include "%s"\n'
                   % os.path.join(root, "reacherdistilation_amd", "csrc", "rd_crc32c.cpp"))
    subprocess.run([gxx, "-O2", "-shared", "-fPIC", "-o", so, str(src)], check=True)
    fn = ctypes.CDLL(so).rd_crc32c
    fn.restype, fn.argtypes = ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_int64, ctypes.c_uint32]
    d = np.random.RandomState(1).randint(0, 256, 200_000).astype(np.uint8).tobytes()
    for n in list(range(71)) + [len(d)]:
        assert fn(d[:n], n, 0) == tc.crc32c_py(d[:n]) == tc.crc32c(d[:n]), n
    assert fn(d[77:], len(d) - 77, fn(d[:77], 77, 0)) == tc.crc32c(d)

def test_lstm_checkpoint_round_trip_is_fast(tmp_path):
    """a T = 10 LSTM checkpoint with its Adam slots (6.1 MB) is written and read back
    (every CRC checked) in well under a second -- lstm_train saves one every episode."""
    import time
    T = 10
    P = tc.lstm_variables(T)
    n = sum(int(np.prod(shape)) for _, _, shape in P)
    rs = np.random.RandomState(1)
    p, m, v = (rs.standard_normal(n).astype(np.float32) for _ in range(3))
    t0 = time.perf_counter()
    tc.save_lstm(str(tmp_path / "lstm.ckpt"), p, m, v, T)
    q, qm, qv = tc.load_lstm(str(tmp_path / "lstm.ckpt"), T)
    el = time.perf_counter() - t0
    assert np.array_equal(q, p) and np.array_equal(qm, m) and np.array_equal(qv, v)
    assert el < 0.5, el


def _tensors(rs):
    return {
        "a/kernel": rs.standard_normal((11, 64)).astype(np.float32),
        "a/bias": rs.standard_normal(64).astype(np.float32),
        "b/count": np.array(123456.5, np.float64),
        "b/sum": rs.standard_normal(11),
        "c/steps": np.array([3, -7, 1 << 40], np.int64),
        "c/i32": np.arange(-5, 5, dtype=np.int32).reshape(2, 5),
        "d/flag": np.array([True, False, True]),
        "d/half": rs.standard_normal(7).astype(np.float16),
        "e/empty": np.zeros((0, 3), np.float32),
    }


def test_round_trip_every_dtype_and_shape(tmp_path):
    t = _tensors(np.random.RandomState(0))
    pre = str(tmp_path / "model.ckpt")
    tc.write(pre, t)
    back = tc.read(pre)
    assert sorted(back) == sorted(t)
    for k, v in t.items():
        assert back[k].dtype == v.dtype and back[k].shape == v.shape, k
        assert back[k].tobytes() == v.tobytes(), k


def test_many_keys_span_several_table_blocks(tmp_path):
    """> 4 KiB of index entries: several data blocks behind the index block, prefix-compressed
    keys with restarts every 16 entries."""
    rs = np.random.RandomState(1)
    t = {f"scope_{i // 40:03d}/layer_{i:04d}/kernel_with_a_long_name": rs.standard_normal(3).astype(np.float32)
         for i in range(400)}
    pre = str(tmp_path / "big.ckpt")
    tc.write(pre, t)
    buf = open(pre + ".index", "rb").read()
    idx = list(tc._read_table(buf))
    assert [k for k, _ in idx] == sorted(k for k, _ in idx) and idx[0][0] == b""
    f = buf[-tc._FOOTER:-8]
    _, i = tc._read_uvarint(f, 0)
    _, i = tc._read_uvarint(f, i)
    io, i = tc._read_uvarint(f, i)
    isz, _ = tc._read_uvarint(f, i)
    assert len(list(tc._block_entries(tc._read_block(buf, io, isz)))) > 1
    back = tc.read(pre)
    assert all(np.array_equal(back[k], v) for k, v in t.items())


def test_format_invariants(tmp_path):
    pre = str(tmp_path / "m.ckpt")
    tc.write(pre, {"x": np.arange(4, dtype=np.float32)})
    buf = open(pre + ".index", "rb").read()
    lo, hi = struct.unpack_from("<II", buf, len(buf) - 8)
    assert (hi << 32 | lo) == 0xDB4775248B80FB57
    rows = dict(tc._read_table(buf))
    h = tc._parse_header(rows[b""])
    assert h == dict(num_shards=1, endianness=0, producer=1)
    e = tc._parse_entry(rows[b"x"])
    assert (e["dtype"], e["shape"], e["shard_id"], e["offset"], e["size"]) == (1, (4,), 0, 0, 16)
    raw = open(pre + ".data-00000-of-00001", "rb").read()
    assert raw == np.arange(4, dtype="<f4").tobytes()
    assert tc._unmask(e["crc32c"]) == tc.crc32c(raw)


def test_corruption_is_detected(tmp_path):
    pre = str(tmp_path / "m.ckpt")
    tc.write(pre, {"x": np.arange(8, dtype=np.float32)})
    d = bytearray(open(pre + ".data-00000-of-00001", "rb").read())
    d[5] ^= 1
    open(pre + ".data-00000-of-00001", "wb").write(bytes(d))
    with pytest.raises(ValueError, match="checksum"):
        tc.read(pre)
    tc.write(pre, {"x": np.arange(8, dtype=np.float32)})
    b = bytearray(open(pre + ".index", "rb").read())
    b[3] ^= 0x40
    open(pre + ".index", "wb").write(bytes(b))
    with pytest.raises(ValueError):
        tc.read(pre)


@pytest.fixture(scope="module")
def ref_graph():
    from oracle import tfgraph
    try:
        return tfgraph.reference_graph()[0]
    except FileNotFoundError:
        pytest.skip("reference event files not present")


def test_teacher_variables_are_the_reference_savers(ref_graph):
    """The reference teacher's Saver (save/SaveV2 of its logged GraphDef) saves exactly the
    variables TEACHER_VARS lists, with the VariableV2 shapes and dtypes given there."""
    nodes = ref_graph.nodes
    saved = nodes["save/SaveV2"]["inputs"][3:]
    assert saved == sorted(n for n, _, _ in tc.TEACHER_VARS)
    dt = {1: np.float32, 2: np.float64}
    for n, shape, d in tc.TEACHER_VARS:
        v = nodes[n]
        assert v["op"] == "VariableV2"
        assert tuple(v["attr"]["shape"][1]) == shape, n
        assert dt[v["attr"]["dtype"][1]] == d, n


def test_obfilter_restore_matches_the_reference_graph(ref_graph):
    """mean / std the restored filter yields, against the graph's pi/obfilter ops evaluated on
    the same variable values (one feature below the 1e-2 variance floor)."""
    rs = np.random.RandomState(3)
    c = 5000.0
    mean = rs.uniform(-1, 1, 11)
    var = rs.uniform(0.02, 4, 11)
    var[4] = 1e-3
    s, q = mean * c, (var + mean * mean) * c
    feeds = {"pi/obfilter/runningsum": s, "pi/obfilter/runningsumsq": q, "pi/obfilter/count": np.float64(c)}
    g_mean, g_std = ref_graph.run(["pi/obfilter/ToFloat", "pi/obfilter/Sqrt"], feeds)
    m, sd = tc.obfilter(s, q, c)
    np.testing.assert_allclose(m, g_mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(sd, g_std, rtol=1e-6)
    assert sd[4] == pytest.approx(0.1, rel=1e-6)


def test_teacher_round_trip_and_teacher_agent(tmp_path):
    p = synthetic_teacher(7)
    p.ob_mean[:] = np.random.RandomState(1).uniform(-.5, .5, 11).astype(np.float32)
    p.ob_std[:] = np.random.RandomState(2).uniform(.2, 3, 11).astype(np.float32)
    pre = str(tmp_path / "teacher.ckpt")
    vf = {"pi/vf/final/bias": np.array([0.25], np.float32)}
    tc.save_teacher(pre, p, vf=vf)
    raw = tc.read(pre)
    assert sorted(raw) == sorted(n for n, _, _ in tc.TEACHER_VARS)
    assert raw["pi/vf/final/bias"][0] == np.float32(0.25)
    q = tc.load_teacher(pre)
    assert np.array_equal(q.flat, p.flat)
    np.testing.assert_allclose(q.ob_mean, p.ob_mean, rtol=0, atol=1e-7)
    np.testing.assert_allclose(q.ob_std, p.ob_std, rtol=1e-6)
    agent = TeacherAgent(restore=True, path=pre)      # reference teacher.py:19-20
    assert np.array_equal(agent.pi.flat, p.flat)


def test_load_teacher_rejects_other_checkpoints(tmp_path):
    pre = str(tmp_path / "lstm.ckpt")
    tc.write(pre, {"LSTM/unique_lstm_cell/kernel": np.zeros((14, 4), np.float32)})
    with pytest.raises(KeyError, match="missing"):
        tc.load_teacher(pre)
    with pytest.raises(ValueError, match="floor"):
        tc.save_teacher(str(tmp_path / "t.ckpt"), MlpPolicyParams(np.zeros(5060, np.float32), np.zeros(11, np.float32),
                                                                  np.full(11, 0.01, np.float32)))


def test_lstm_saver_layout_matches_the_reference_graph(ref_graph):
    """The reference's 'LSTM'-scope Saver (save_1/SaveV2 of its logged GraphDef, an older
    per-step-named variant of student_lstm_graph) saves every variable of the scope together
    with its '/Adam' and '/Adam_1' slots and nothing else; the cell is 'unique_lstm_cell'.
    save_lstm writes the same structure for the current graph."""
    nodes = ref_graph.nodes
    saved = nodes["save_1/SaveV2"]["inputs"][3:]
    lstm = sorted(n for n, v in nodes.items() if v["op"] == "VariableV2" and n.startswith("LSTM/"))
    assert saved == lstm
    base = [n for n in lstm if not n.endswith(("/Adam", "/Adam_1"))]
    assert sorted(b + s for b in base for s in ("", "/Adam", "/Adam_1")) == lstm
    assert "LSTM/unique_lstm_cell/kernel" in base
    names = {n for n, _, _ in tc.lstm_variables(10)}
    assert "LSTM/unique_lstm_cell/kernel" in names and "LSTM/unique_lstm_cell/bias" in names


def test_lstm_round_trip(tmp_path):
    from reacherdistilation_amd import student_lstm as sl
    T = 3
    n = sl.n_params(T)
    rs = np.random.RandomState(5)
    p, m, v = (rs.standard_normal(n).astype(np.float32) for _ in range(3))
    pre = str(tmp_path / "lstm_with_keep_probability_1.0.ckpt")
    tc.save_lstm(pre, p, m, v, T)
    raw = tc.read(pre)
    var = tc.lstm_variables(T)
    assert len(var) == 4 + 10 * T and len(raw) == 3 * len(var)
    assert raw["LSTM/unique_lstm_cell/kernel"].shape == (243, 800)
    assert raw["LSTM/dense_15/bias"].shape == (4,)        # step 2's output layer (calls 11 .. 15)
    o = dict((k, (off, s)) for k, off, s in var)["LSTM/dense_6/kernel"]   # step 1's first layer
    assert np.array_equal(raw["LSTM/dense_6/kernel"].ravel(), p[o[0]:o[0] + 200 * 64])
    q, qm, qv = tc.load_lstm(pre, T)
    assert np.array_equal(q, p) and np.array_equal(qm, m) and np.array_equal(qv, v)
    tc.save_lstm(pre, p, T=T)                              # no slots: parameters only
    q, qm, qv = tc.load_lstm(pre, T)
    assert np.array_equal(q, p) and qm is None and qv is None
    with pytest.raises(KeyError, match="missing"):
        tc.load_lstm(pre, T + 1)
