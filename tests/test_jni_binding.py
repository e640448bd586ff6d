"""The Java shim's JNI binding (java/jni/scotty_jni.c) executed end to end, without a JDK: the binding and a
functional mock JNIEnv (tests/jni_mock/mock_jni.c: arrays, direct ByteBuffers, the NativeApi.Windows object, field
lookup by name and signature, local-reference and pending-exception accounting) are linked into
tests/jni_mock/libjni_mock.so, and this test calls the JNI entry points exactly as the Java shim does:

* ``JniOp`` mirrors the stand-alone mode of java/main/.../SlicingWindowOperator.java: processElement appends to
  off-heap direct buffers (here numpy arrays wrapped by the mock's direct ByteBuffer), the buffer goes to the GPU as
  one micro-batch (processElements0) before processWatermark0 fills a NativeApi.Windows object;
* ``JniKeyedEngine`` mirrors java/main/.../KeyedEngine.java: one keyed native operator, (id, ts, value) micro-batches
  through processKeyedElements0, one processWatermark0 per round, rows grouped by the key column.

Rows are compared bit-exactly with the CPU oracle (GlobalScottyWindowOperator / KeyedScottyWindowOperator semantics:
F/GlobalScottyWindowOperator.java:40-64, F/KeyedScottyWindowOperator.java:56-86).  The CPU tests check the binding's
argument handling that needs no device (heap buffers, library symbols)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from helpers import ROOT, product, same_windows, KeyedOracle, same_keyed_windows
from specs import Tumbling, Sliding, Session, Time, SUM, COUNT, MIN, MAX

MOCK_DIR = os.path.join(ROOT, "tests", "jni_mock")
MOCK_LIB = os.path.join(MOCK_DIR, "libjni_mock.so")
P, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
PKG = "Java_de_tub_dima_scotty_slicing_JniApi_"
# JniApi.java's native methods: (restype, argtypes after (JNIEnv*, jclass))
NATIVES = {
    "create0": (i64, [i32, i32, i32, P]),
    "destroy0": (None, [i64]),
    "lastError0": (P, [i64]),
    "addWindow0": (i32, [i64, i32, i32, i64, i64]),
    "addAggregation0": (i32, [i64, i32]),
    "setMaxLateness0": (i32, [i64, i64]),
    "processElements0": (i32, [i64, P, P, i64]),
    "processKeyedElements0": (i32, [i64, P, P, P, i64]),
    "processWatermark0": (i32, [i64, i64, P]),
    "firstIndices0": (P, [i64]),
}
M_LONGS, M_INTS, M_BYTES, M_OBJS, M_STRING = 5, 6, 7, 8, 2

_mock = None


def mock():
    """libjni_mock.so (built by tests/jni_mock/Makefile against the in-tree product library)."""
    global _mock
    if _mock is None:
        product().lib()  # the product library first (the mock links it by rpath: the same file)
        if not os.path.exists(MOCK_LIB):
            subprocess.check_call(["make", "-s", "-C", MOCK_DIR])
        L = ctypes.CDLL(MOCK_LIB)
        for name, (res, args) in NATIVES.items():
            f = getattr(L, PKG + name)
            f.restype, f.argtypes = res, [P, P] + args
        for name, res, args in [("mock_env", P, []), ("mock_direct_buffer", P, [P, i64]), ("mock_heap_buffer", P, []),
                                ("mock_int_array", P, [i32]), ("mock_windows", P, []), ("mock_windows_n", i32, [P]),
                                ("mock_windows_field", P, [P, ctypes.c_int]), ("mock_kind", ctypes.c_int, [P]),
                                ("mock_length", i32, [P]), ("mock_data", P, [P]), ("mock_element", P, [P, i32]),
                                ("mock_local_refs", ctypes.c_int, []), ("mock_exceptions", ctypes.c_int, []),
                                ("mock_last_exception", ctypes.c_char_p, []), ("mock_reset", None, [])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _mock = L
    return _mock


def jni(name, *args):
    L = mock()
    return getattr(L, PKG + name)(L.mock_env(), None, *args)


def _array(L, obj, dtype):
    n = L.mock_length(obj)
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ctypes.cast(L.mock_data(obj), ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                 shape=(n,)).copy()


def read_windows(w):
    """NativeApi.Windows as the shim reads it: n, start, end, measure, has, values[n_aggs][n], key (or null)."""
    L = mock()
    n = L.mock_windows_n(w)
    f = [L.mock_windows_field(w, k) for k in range(6)]
    kinds = [L.mock_kind(x) for x in f]
    assert kinds[:5] == [M_LONGS, M_LONGS, M_INTS, M_BYTES, M_OBJS], kinds
    start, end = _array(L, f[0], np.int64), _array(L, f[1], np.int64)
    measure, has = _array(L, f[2], np.int32), _array(L, f[3], np.int8)
    assert len(start) == len(end) == len(measure) == len(has) == n
    values = [_array(L, L.mock_element(f[4], k), np.int64) for k in range(L.mock_length(f[4]))]
    assert all(len(v) == n for v in values)
    key = _array(L, f[5], np.int32) if f[5] else None
    return n, start, end, measure, has, values, key


def rows_of(win, lo=None, hi=None):
    """AggregateWindows (the shim's NativeAggregateWindow before lower()) of rows [lo, hi)."""
    pkg = product()
    n, start, end, measure, has, values, _ = win
    rng = range(n) if lo is None else range(lo, hi)
    return [pkg.AggregateWindow(int(start[i]), int(end[i]), int(measure[i]), bool(has[i]),
                                [int(v[i]) for v in values] if has[i] else []) for i in rng]


class JniOp:
    """The stand-alone mode of java/main/.../SlicingWindowOperator.java over the JNI entry points."""

    def __init__(self, cfg, value_type=0, device=0):
        L = mock()
        rc = L.mock_int_array(1)  # `new int[1]`
        self.op = jni("create0", device, value_type, 0, rc)
        assert self.op != 0, "create0 rc %d" % _array(L, rc, np.int32)[0]
        for a in cfg["aggs"]:
            self.check(jni("addAggregation0", self.op, a))
        if cfg.get("lateness") is not None:
            self.check(jni("setMaxLateness0", self.op, cfg["lateness"]))
        for w in cfg["windows"]:
            self.check(jni("addWindow0", self.op, w.kind, w.measure, w.a, w.b))
        self.ts, self.vals = [], []  # the off-heap micro-batch (tsBuf / valBuf)

    def check(self, rc):
        if rc < 0:
            s = jni("lastError0", self.op)
            raise RuntimeError("rc %d: %s" % (rc, ctypes.string_at(mock().mock_data(s)).decode()))
        return rc

    def processElements(self, ts, vals):
        self.ts.append(np.asarray(ts, dtype=np.int64))
        self.vals.append(np.asarray(vals, dtype=np.int32))

    def flush(self):
        if not self.ts:
            return
        ts, v = np.ascontiguousarray(np.concatenate(self.ts)), np.ascontiguousarray(np.concatenate(self.vals))
        self.ts, self.vals = [], []
        L = mock()
        bt, bv = L.mock_direct_buffer(ts.ctypes.data, ts.nbytes), L.mock_direct_buffer(v.ctypes.data, v.nbytes)
        self.check(jni("processElements0", self.op, bt, bv, len(ts)))

    def processWatermark(self, wm):
        self.flush()
        L = mock()
        w = L.mock_windows()  # new NativeApi.Windows()
        refs = L.mock_local_refs()
        self.check(jni("processWatermark0", self.op, wm, w))
        assert L.mock_exceptions() == 0, L.mock_last_exception()
        # every array the binding made is either stored in a field or released; what is left is the class references
        # (GetObjectClass, FindClass), which the JVM reclaims at return
        assert L.mock_local_refs() - refs <= 2, L.mock_local_refs() - refs
        return rows_of(read_windows(w))

    def close(self):
        jni("destroy0", self.op)


# ------------------------------------------------------------------------------------------------------------ CPU
def test_mock_library_exports_every_native_method():
    L = mock()
    for name in NATIVES:
        assert getattr(L, PKG + name) is not None


def test_heap_buffers_are_refused_before_the_library():
    """processElements0 / processKeyedElements0 with a heap ByteBuffer (no direct address): SCOTTY_ERR_ARG from the
    binding itself (java/jni/scotty_jni.c), no library call -- so op = 0 is never dereferenced."""
    L = mock()
    h = L.mock_heap_buffer()
    assert jni("processElements0", 0, h, h, 5) == -1
    assert jni("processKeyedElements0", 0, h, h, h, 5) == -1
    assert L.mock_exceptions() == 0


# ------------------------------------------------------------------------------------------------------------ GPU
def _stream(n, seed, ooo=0.2, delay=300, rate=20, t0=10):
    rng = np.random.default_rng(seed)
    ts = t0 + np.arange(n, dtype=np.int64) // rate
    late = rng.random(n) < ooo
    ts = np.where(late, np.maximum(ts - rng.integers(1, delay + 1, n), 1), ts)
    vals = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    return ts, vals


CFGS = {
    "grid_sliding_tumbling": dict(windows=[Sliding(Time, 1000, 100), Tumbling(Time, 700)], aggs=[SUM, COUNT, MIN],
                                  lateness=1000),
    "exact_session": dict(windows=[Sliding(Time, 2000, 250), Session(Time, 150)], aggs=[SUM, COUNT, MIN, MAX],
                          lateness=1000),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CFGS))
def test_jni_operator_matches_oracle(name):
    from oracle.oracle import OracleOperator
    cfg = CFGS[name]
    op = JniOp(cfg)
    ora = OracleOperator()
    for a in cfg["aggs"]:
        ora.addWindowFunction(a)
    ora.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        ora.addWindowAssigner(w)
    ts, vals = _stream(120_000, seed=len(name))
    total = 0
    for lo in range(0, len(ts), 20_000):
        hi = lo + 20_000
        for a in range(lo, hi, 5_000):  # several processElement runs per micro-batch (one off-heap buffer)
            op.processElements(ts[a:a + 5_000], vals[a:a + 5_000])
        assert ora.processElements(ts[lo:hi], vals[lo:hi]) == 0
        wm = int(ts[:hi].max()) - 300
        got, exp = op.processWatermark(wm), ora.processWatermark(wm)
        same_windows(got, exp)
        total += len(exp)
    assert total > 10  # (6 s of event time: ~20 sliding windows per config)
    op.close()
    mock().mock_reset()


@pytest.mark.gpu
def test_jni_errors_come_back_as_status_and_message():
    """An unknown aggregation kind: the binding returns the library's status, lastError0 carries its message as a
    Java string (the shim throws UnsupportedOperationException with it)."""
    L = mock()
    op = JniOp(dict(windows=[Tumbling(Time, 100)], aggs=[SUM], lateness=10))
    rc = jni("addAggregation0", op.op, 0x7777)
    assert rc < 0
    s = jni("lastError0", op.op)
    assert L.mock_kind(s) == M_STRING and len(ctypes.string_at(L.mock_data(s))) > 0
    op.close()
    L.mock_reset()


class JniKeyedEngine:
    """java/main/.../KeyedEngine.java over the JNI entry points: one keyed native op, one push + one watermark per
    round, rows grouped by the key column."""

    def __init__(self, cfg):
        L = mock()
        rc = L.mock_int_array(1)
        self.op = jni("create0", 0, 0, 1, rc)  # FLAG_KEYED
        assert self.op != 0
        for w in cfg["windows"]:
            assert jni("addWindow0", self.op, w.kind, w.measure, w.a, w.b) >= 0
        for a in cfg["aggs"]:
            assert jni("addAggregation0", self.op, a) >= 0
        if cfg.get("lateness") is not None:
            assert jni("setMaxLateness0", self.op, cfg["lateness"]) >= 0

    def push(self, keys, ts, vals):
        L = mock()
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        v = np.ascontiguousarray(vals, dtype=np.int32)
        bk, bt, bv = (L.mock_direct_buffer(x.ctypes.data, x.nbytes) for x in (k, t, v))
        assert jni("processKeyedElements0", self.op, bk, bt, bv, len(t)) >= 0

    def watermark(self, wm):
        L = mock()
        w = L.mock_windows()
        assert jni("processWatermark0", self.op, wm, w) >= 0
        assert L.mock_exceptions() == 0, L.mock_last_exception()
        win = read_windows(w)
        assert win[6] is not None and len(win[6]) == win[0]  # keyed: the key column is set
        rows = rows_of(win)
        return [(int(win[6][i]), rows[i]) for i in range(win[0])]


@pytest.mark.gpu
def test_jni_keyed_engine_matches_per_key_oracles():
    cfg = dict(windows=[Sliding(Time, 1000, 250), Tumbling(Time, 500)], aggs=[SUM, COUNT], lateness=500)
    eng = JniKeyedEngine(cfg)
    ora = KeyedOracle(cfg)
    rng = np.random.default_rng(3)
    nkeys, n = 2000, 200_000
    t = 0
    total = 0
    for step in range(4):
        keys = rng.integers(0, nkeys, n).astype(np.uint32)
        ts = t + np.sort(rng.integers(0, 1000, n)).astype(np.int64)
        vals = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        eng.push(keys, ts, vals)
        ora.processElements(keys, ts, vals)
        wm = t + 999
        total += same_keyed_windows(eng.watermark(wm), ora.processWatermark(wm))
        t += 1000
    assert total > nkeys
    jni("destroy0", eng.op)
    mock().mock_reset()


class JniFirstShim(JniOp):
    """The stand-alone shim with a first-partial function (java/main/.../SlicingWindowOperator.java, NativeFunctions
    TUPLE2_F1 / TUPLE4_F1): the hidden SCOTTY_AGG_FIRST column after the function's, the payloads of this interval's
    tuples plus the retained slices' first tuples (firstIndices0 after every watermark), and each window's result
    rebuilt from the payload of its first partial's tuple."""

    def __init__(self, cfg, payload):
        super().__init__(dict(cfg, aggs=list(cfg["aggs"]) + [10]))
        self.payload = payload          # arrival index -> the tuple's other fields (the Java objects)
        self.arrivals = self.base = 0
        self.retained = {}

    def processElements(self, ts, vals):
        super().processElements(ts, vals)
        self.arrivals += len(ts)

    def fields(self, i):
        if i >= self.base:
            assert i < self.arrivals, (i, self.arrivals)
            return self.payload(i)
        assert i in self.retained, ("first tuple %d was pruned" % i)
        return self.retained[i]

    def processWatermark(self, wm):
        rows = super().processWatermark(wm)
        out = []
        for w in rows:
            if w.hasValue():
                v = w.getAggValues()
                out.append((w.getStart(), w.getEnd(), v[:-1], self.fields(v[-1])))
            else:
                out.append((w.getStart(), w.getEnd(), [], None))
        L = mock()
        arr = jni("firstIndices0", self.op)
        assert arr, "firstIndices0 returned null"
        keep = _array(L, arr, np.int64)
        self.retained = {int(i): self.fields(int(i)) for i in keep}
        self.base = self.arrivals
        return out


def _first_rows(ora_rows, payload):
    return [(w.getStart(), w.getEnd(), w.getAggValues()[:-1] if w.hasValue() else [],
             payload(w.getAggValues()[-1]) if w.hasValue() else None) for w in ora_rows]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["benchmark_tuple4_c1", "flink_demo_tuple2_varying_f0"])
def test_jni_first_partial_rebuild_matches_oracle(case):
    """the reference benchmark's SumAggregation (Tuple4 f0 / f2 / f3 of the first partial) on the C1
    stream, and the Flink demo's SumWindowFunction (Tuple2 f0) under GlobalScottyWindowOperator with f0 varying from
    tuple to tuple and 20 % late tuples: every window's rebuilt result equals the one the oracle's first-partial index
    selects, and every needed payload was still held (retained firsts + this interval's tuples)."""
    from oracle.oracle import OracleOperator, AGG_FIRST
    rng = np.random.default_rng(606)
    if case == "benchmark_tuple4_c1":
        cfg = dict(windows=[Sliding(Time, 60_000, 1000)], aggs=[SUM], lateness=1)
        rate, secs = 20, 75
        ts = np.arange(secs * 1000 * rate, dtype=np.int64) // rate
        vals = product().workloads.JavaRandomInts(43).next_ints(len(ts))
        f2 = rng.integers(-2**63, 2**63 - 1, len(ts), dtype=np.int64)  # LoadGeneratorSource: nextLong, currentTimeMillis
        payload = lambda i: ("key", int(f2[i]), int(ts[i]) + 1_700_000_000_000)  # noqa: E731
        cuts = [(s * 1000 * rate, (s + 1) * 1000 * rate, s * 1000 + 999) for s in range(secs)]
    else:
        cfg = dict(windows=[Tumbling(Time, 700), Sliding(Time, 2000, 300)], aggs=[SUM], lateness=1000)
        ts, vals = _stream(150_000, seed=9, ooo=0.2, delay=400, rate=20)
        f0 = rng.integers(0, 1000, len(ts))
        payload = lambda i: (int(f0[i]),)  # noqa: E731
        cuts = [(lo, lo + 15_000, int(ts[:lo + 15_000].max()) - 400) for lo in range(0, len(ts), 15_000)]
    shim = JniFirstShim(cfg, payload)
    ora = OracleOperator()
    for a in cfg["aggs"] + [AGG_FIRST]:
        ora.addWindowFunction(a)
    ora.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        ora.addWindowAssigner(w)
    total = 0
    for lo, hi, wm in cuts:
        shim.processElements(ts[lo:hi], vals[lo:hi])
        ora.processElements(ts[lo:hi], vals[lo:hi])
        got, exp = shim.processWatermark(wm), _first_rows(ora.processWatermark(wm), payload)
        assert got == exp
        total += sum(1 for r in exp if r[3] is not None)
    assert total > 10
    shim.close()
    mock().mock_reset()
