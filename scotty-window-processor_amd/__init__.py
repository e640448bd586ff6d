"""Python host mirror of the reference operator API over the MI355X C-ABI (include/scotty_mi355x.h).

Same names, argument meaning and error behaviour as the reference
(core/src/main/java/de/tub/dima/scotty/core/WindowOperator.java:9-40 and
slicing/src/main/java/de/tub/dima/scotty/slicing/SlicingWindowOperator.java:21-69):

    op = SlicingWindowOperator()
    op.addWindowFunction(SumAggregateFunction())          # or the integer kind SCOTTY_AGG_SUM_I32
    op.addWindowAssigner(TumblingWindow(WindowMeasure.Time, 10))
    op.processElement(1, 1)
    for w in op.processWatermark(22): w.getStart(), w.getEnd(), w.getAggValues(), w.hasValue()

processElement() calls are buffered host-side (as the JVM shim buffers them off-heap) and handed to the
GPU as one micro-batch; processElements()/processElementsDevice() hand over whole batches.  There is no
CPU fallback: if libscotty_mi355x.so cannot be loaded or no GPU is present, construction raises.
"""
import ctypes
import os
import struct

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libscotty_mi355x.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "scotty_mi355x.h")

SCOTTY_OK, SCOTTY_WARN_LATE_DROPPED = 0, 1
FLAG_KEYED = 0x1
ERRORS = {-1: "SCOTTY_ERR_ARG", -2: "SCOTTY_ERR_UNSUPPORTED", -3: "SCOTTY_ERR_HIP", -4: "SCOTTY_ERR_STATE",
          -5: "SCOTTY_ERR_INDEX", -6: "SCOTTY_ERR_NOMEM"}
VALUE_I32, VALUE_I64, VALUE_F64 = 0, 1, 2
AGG_SUM_I32, AGG_COUNT, AGG_MIN_I32, AGG_MAX_I32 = 0, 1, 2, 3
AGG_SUM_I64, AGG_MIN_I64, AGG_MAX_I64 = 4, 5, 6
AGG_SUM_F64, AGG_MIN_F64, AGG_MAX_F64 = 7, 8, 9
# the arrival index of the window's first partial (include/scotty_mi355x.h SCOTTY_AGG_FIRST): what a combine keeping
# partialAggregate1's fields returns (B/flinkBenchmark/aggregations/SumAggregation.java:16-18); grid path only
AGG_FIRST = 10
F64_AGGS = (AGG_SUM_F64, AGG_MIN_F64, AGG_MAX_F64)
AGG_INVERTIBLE = 0x10000  # OR-able: the function is an InvertibleAggregateFunction (include/scotty_mi355x.h)
MAX_AGGS = 8


class ScottyError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (ERRORS.get(code, code), msg))
        self.code = code


class UnsupportedError(ScottyError):
    pass


class WindowMeasure:  # C/windowType/WindowMeasure.java
    Time = 0
    Count = 1


class _Window:
    kind = -1

    def __init__(self, measure, a, b=0):
        self.measure, self.a, self.b = measure, a, b


class TumblingWindow(_Window):  # C/windowType/TumblingWindow.java
    kind = 0

    def __init__(self, measure, size):
        super().__init__(measure, size)


class SlidingWindow(_Window):  # C/windowType/SlidingWindow.java
    kind = 1

    def __init__(self, measure, size, slide):
        super().__init__(measure, size, slide)


class SessionWindow(_Window):  # C/windowType/SessionWindow.java
    kind = 2

    def __init__(self, measure, gap):
        super().__init__(measure, gap)


class FixedBandWindow(_Window):  # C/windowType/FixedBandWindow.java
    kind = 3

    def __init__(self, measure, start, size):
        super().__init__(measure, start, size)


class _Agg:  # known AggregateFunction classes the GPU path recognises (C/windowFunction/)
    kind = -1


def _agg(kind_, name):
    return type(name, (_Agg,), {"kind": kind_})


SumAggregateFunction = _agg(AGG_SUM_I32, "SumAggregateFunction")
CountAggregateFunction = _agg(AGG_COUNT, "CountAggregateFunction")
MinAggregateFunction = _agg(AGG_MIN_I32, "MinAggregateFunction")
MaxAggregateFunction = _agg(AGG_MAX_I32, "MaxAggregateFunction")
LongSumAggregateFunction = _agg(AGG_SUM_I64, "LongSumAggregateFunction")
DoubleSumAggregateFunction = _agg(AGG_SUM_F64, "DoubleSumAggregateFunction")
# InvertibleReduceAggregateFunction variants (C/windowFunction/InvertibleReduceAggregateFunction.java)
InvertibleSumAggregateFunction = _agg(AGG_SUM_I32 | AGG_INVERTIBLE, "InvertibleSumAggregateFunction")
InvertibleCountAggregateFunction = _agg(AGG_COUNT | AGG_INVERTIBLE, "InvertibleCountAggregateFunction")


class scotty_windows(ctypes.Structure):
    _fields_ = [("n_windows", ctypes.c_size_t), ("n_aggs", ctypes.c_int32),
                ("start", ctypes.POINTER(ctypes.c_int64)), ("end", ctypes.POINTER(ctypes.c_int64)),
                ("measure", ctypes.POINTER(ctypes.c_int32)), ("has_value", ctypes.POINTER(ctypes.c_uint8)),
                ("values", ctypes.POINTER(ctypes.c_int64) * MAX_AGGS),
                ("key", ctypes.POINTER(ctypes.c_uint32))]


_lib = None


def header_functions():
    """Function names declared by include/scotty_mi355x.h."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|void\*|const char\*|uint64_t|int64_t|int32_t)\s+(scotty_\w+)\(", txt, re.M)))


def _single_hip_runtime():
    """True when exactly one libamdhip64 is mapped into this process (after the library is loaded): the library
    and torch then share one HIP runtime, and their streams and events can order each other."""
    lib()
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if os.path.basename(p).startswith("libamdhip64.so"):
                paths.add(os.path.realpath(p))
    return len(paths) == 1


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libscotty_mi355x.so not built (run __graft_entry__.build()): " + LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        P, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
        sig = {
            "scotty_create": (ctypes.c_int, [ctypes.POINTER(P), ctypes.c_int, ctypes.c_int, ctypes.c_uint32]),
            "scotty_destroy": (None, [P]),
            "scotty_last_error": (ctypes.c_char_p, [P]),
            "scotty_add_window": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, i64, i64]),
            "scotty_add_aggregation": (ctypes.c_int, [P, ctypes.c_int]),
            "scotty_set_max_lateness": (ctypes.c_int, [P, i64]),
            "scotty_process_elements": (ctypes.c_int, [P, P, P, ctypes.c_size_t]),
            "scotty_process_elements_device": (ctypes.c_int, [P, P, P, ctypes.c_size_t]),
            "scotty_process_watermark": (ctypes.c_int, [P, i64, ctypes.POINTER(scotty_windows)]),
            "scotty_process_watermark_device": (ctypes.c_int, [P, i64, ctypes.POINTER(scotty_windows)]),
            "scotty_process_keyed_elements": (ctypes.c_int, [P, P, P, P, ctypes.c_size_t]),
            "scotty_process_keyed_elements_device": (ctypes.c_int, [P, P, P, P, ctypes.c_size_t]),
            "scotty_key_count": (i64, [P]),
            "scotty_tune": (ctypes.c_int, [P, ctypes.c_char_p, i64]),
            "scotty_shard_xbytes": (ctypes.c_size_t, [P]),
            "scotty_shard_push": (ctypes.c_int, [P, P, P, ctypes.c_size_t, i64, P]),
            "scotty_shard_commit": (ctypes.c_int, [P, P, ctypes.c_int]),
            "scotty_shard_push_counted": (ctypes.c_int, [P, P, P, ctypes.c_size_t, i64, i64, i64, P]),
            "scotty_shard_push_timed": (ctypes.c_int, [P, P, P, ctypes.c_size_t, i64, i64, i64, i64, i64, P]),
            "scotty_shard_bounds": (ctypes.c_int, [P, P, ctypes.c_size_t, P]),
            "scotty_dropped_count": (u64, [P]),
            "scotty_processed_count": (u64, [P]),
            "scotty_slice_count": (i64, [P]),
            "scotty_first_indices": (i64, [P, P, ctypes.c_size_t]),
            "scotty_enable_timing": (ctypes.c_int, [P, ctypes.c_int]),
            "scotty_ingest_timing": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64),
                                                    ctypes.POINTER(u64)]),
            "scotty_device_timing": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(u64)]),
            "scotty_sync": (ctypes.c_int, [P]),
            "scotty_key_shard": (ctypes.c_int32, [ctypes.c_uint32, ctypes.c_int, ctypes.c_int]),
            "scotty_stream_order": (ctypes.c_int, [P, P, ctypes.c_int]),
            "scotty_op_stream": (P, [P]),
            "scotty_route_keyed": (ctypes.c_int, [P, P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int, P, P, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


class AggregateWindow:  # C/AggregateWindow.java:8-21
    __slots__ = ("start", "end", "measure", "_has", "_values")

    def __init__(self, start, end, measure, has, values):
        self.start, self.end, self.measure, self._has, self._values = start, end, measure, has, values

    def getStart(self):
        return self.start

    def getEnd(self):
        return self.end

    def getMeasure(self):
        return self.measure

    def hasValue(self):
        return self._has

    def getAggValues(self):
        return list(self._values)

    def key(self):
        return (self.start, self.end, self.measure, self._has, tuple(self._values))

    def __repr__(self):
        return "AggregateWindow(%d,%d,m=%d,%s)" % (self.start, self.end, self.measure, self._values)


def _kind_of(fn):
    if isinstance(fn, int):
        return fn
    if isinstance(fn, type) and issubclass(fn, _Agg):
        return fn.kind
    if isinstance(fn, _Agg):
        return fn.kind
    raise UnsupportedError(-2, "AggregateFunction %r has no GPU kind (user lambdas cannot run on the GPU)" % (fn,))


class SlicingWindowOperator:
    """de.tub.dima.scotty.slicing.SlicingWindowOperator backed by libscotty_mi355x.so."""

    _flags = 0

    def __init__(self, device=0, value_type=VALUE_I32):
        self._l = lib()
        self._h = ctypes.c_void_p()
        rc = self._l.scotty_create(ctypes.byref(self._h), device, value_type, self._flags)
        if rc != 0:
            raise ScottyError(rc, "scotty_create failed (no MI355X / HIP device?)")
        self.value_type = value_type
        self._aggs = []
        self._buf_ts, self._buf_v = [], []
        self.last_status = 0

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._l.scotty_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            msg = self._l.scotty_last_error(self._h).decode()
            raise (UnsupportedError if rc == -2 else ScottyError)(rc, msg)
        return rc

    def tune(self, key, value):
        """Capacity knobs of the exact engine ("slice_capacity", "session_capacity"), before the first push."""
        self._check(self._l.scotty_tune(self._h, key.encode(), int(value)))

    def _debug_stat(self, which):
        """Internal statistics of the last push (scotty_debug_stat in scotty_engine.cpp); tests and tools only.
        Keyed: 2 path of the last push (0 replay, 1 sort-free, 2 sort-free + replay of deferred keys), 3 deferred
        tuples, 4 keys committed on the sort-free path.  Any operator: 5 engine (1 grid path, 2 exact engine, 3 count
        path), 6 time edges of the count path's last push."""
        f = self._l.scotty_debug_stat
        f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]
        self._flush()
        return int(f(self._h, which))

    # ---- WindowOperator API
    def addWindowAssigner(self, window):
        self._flush()
        self._check(self._l.scotty_add_window(self._h, window.kind, window.measure, window.a, window.b))

    def addAggregation(self, fn):
        self._flush()
        kind = _kind_of(fn)
        idx = self._check(self._l.scotty_add_aggregation(self._h, kind))
        self._aggs.append(kind & 0xFFFF)
        return idx

    addWindowFunction = addAggregation

    def setMaxLateness(self, max_lateness):
        self._flush()
        self._check(self._l.scotty_set_max_lateness(self._h, max_lateness))

    def processElement(self, element, ts):
        self._buf_ts.append(ts)
        self._buf_v.append(element)

    def processElements(self, ts, values):
        """A micro-batch of processElement calls in arrival order (host arrays)."""
        self._flush()
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        dt = {VALUE_I32: np.int32, VALUE_I64: np.int64, VALUE_F64: np.float64}[self.value_type]
        v = np.ascontiguousarray(values, dtype=dt)
        assert len(ts) == len(v)
        if len(ts):
            self._check(self._l.scotty_process_elements(self._h, ts.ctypes.data, v.ctypes.data, len(ts)))

    def hostBuffers(self, n):
        """(ts, values) numpy views of one of the op's two pinned staging slots (scotty_host_buffers) for n tuples:
        fill them and pass them to processElements, which DMAs them in place (no CPU copy).  Slots alternate between
        calls; a slot is handed out again once its previous transfer has finished."""
        self._flush()
        f = self._l.scotty_host_buffers
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]
        pts, pval, pkey = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        self._check(f(self._h, n, ctypes.byref(pts), ctypes.byref(pval), ctypes.byref(pkey)))
        dt = {VALUE_I32: np.int32, VALUE_I64: np.int64, VALUE_F64: np.float64}[self.value_type]
        ts = np.ctypeslib.as_array(ctypes.cast(pts, ctypes.POINTER(ctypes.c_int64)), shape=(n,))
        vals = np.frombuffer((ctypes.c_char * (n * np.dtype(dt).itemsize)).from_address(pval.value), dtype=dt)
        if pkey.value:
            keys = np.ctypeslib.as_array(ctypes.cast(pkey, ctypes.POINTER(ctypes.c_uint32)), shape=(n,))
            return ts, vals, keys
        return ts, vals

    def processElementsDevice(self, ts_ptr, val_ptr, n):
        """A micro-batch already resident in HBM (e.g. torch tensors' data_ptr()); buffers must stay valid
        until the next processWatermark returns."""
        self._flush()
        self._check(self._l.scotty_process_elements_device(self._h, ts_ptr, val_ptr, n))

    def _flush(self):
        if self._buf_ts:
            ts, v = self._buf_ts, self._buf_v
            self._buf_ts, self._buf_v = [], []
            self.processElements(ts, v)

    def processWatermark(self, watermark_ts):
        self._flush()
        out = scotty_windows()
        self.last_status = self._check(self._l.scotty_process_watermark(self._h, watermark_ts, ctypes.byref(out)))
        return self._windows(out)

    def _windows(self, out):
        n = out.n_windows
        res = []
        if n == 0:
            return res
        start = np.ctypeslib.as_array(out.start, shape=(n,)).copy()
        end = np.ctypeslib.as_array(out.end, shape=(n,)).copy()
        meas = np.ctypeslib.as_array(out.measure, shape=(n,)).copy()
        has = np.ctypeslib.as_array(out.has_value, shape=(n,)).copy()
        cols = []
        for k, kind in enumerate(self._aggs):
            col = np.ctypeslib.as_array(out.values[k], shape=(n,)).copy()
            cols.append(col.view(np.float64) if kind in F64_AGGS else col)
        for i in range(n):
            vals = [c[i].item() for c in cols] if has[i] else []
            res.append(AggregateWindow(int(start[i]), int(end[i]), int(meas[i]), bool(has[i]), vals))
        return res

    # ---- time/arrival-range sharding of one non-keyed stream (include/scotty_mi355x.h, scotty_shard_*)
    def shardXBytes(self):
        return self._l.scotty_shard_xbytes(self._h)

    def shardPush(self, ts_ptr, val_ptr, n, ts0, xbuf_ptr):
        self._flush()
        self._check(self._l.scotty_shard_push(self._h, ts_ptr, val_ptr, n, ts0, xbuf_ptr))

    def shardPushCounted(self, ts_ptr, val_ptr, n, ts0, n_before, n_total, xbuf_ptr):
        self._flush()
        self._check(self._l.scotty_shard_push_counted(self._h, ts_ptr, val_ptr, n, ts0, n_before, n_total, xbuf_ptr))

    def shardPushTimed(self, ts_ptr, val_ptr, n, ts0, n_before, n_total, ts_before, ts_last, xbuf_ptr):
        self._flush()
        self._check(self._l.scotty_shard_push_timed(self._h, ts_ptr, val_ptr, n, ts0, n_before, n_total, ts_before,
                                                    ts_last, xbuf_ptr))

    def shardBounds(self, ts_ptr, n):
        """(first, last) timestamp of a device chunk (INT64_MIN for an empty one)."""
        out = (ctypes.c_int64 * 2)()
        self._check(self._l.scotty_shard_bounds(self._h, ts_ptr, n, ctypes.addressof(out)))
        return int(out[0]), int(out[1])

    def streamOrder(self, stream, op_waits):
        """scotty_stream_order: op_waits=False: `stream` (a hipStream_t handle) waits for the op's queued work;
        True: the op's stream waits for the work queued on `stream`."""
        self._check(self._l.scotty_stream_order(self._h, stream, 1 if op_waits else 0))

    def opStream(self):
        """scotty_op_stream: the op's hipStream_t handle (an int)."""
        return int(self._l.scotty_op_stream(self._h) or 0)

    def shardCommit(self, gathered_ptr, world):
        self._check(self._l.scotty_shard_commit(self._h, gathered_ptr, world))

    def processWatermarkDevice(self, watermark_ts):
        """processWatermark with the result columns left in HBM (exact engine): returns (n_windows, status)."""
        self._flush()
        out = scotty_windows()
        st = self._check(self._l.scotty_process_watermark_device(self._h, watermark_ts, ctypes.byref(out)))
        return out.n_windows, st

    def processWatermarkArrays(self, watermark_ts):
        """processWatermark as numpy columns (no per-window objects, for million-window results): a dict with
        start, end, measure, has_value, values (one column per aggregation, registration order) and, on a keyed
        operator, key."""
        self._flush()
        out = scotty_windows()
        self.last_status = self._check(self._l.scotty_process_watermark(self._h, watermark_ts, ctypes.byref(out)))
        n = out.n_windows
        col = lambda p, dt: np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, dt)
        res = {"start": col(out.start, np.int64), "end": col(out.end, np.int64),
               "measure": col(out.measure, np.int32), "has_value": col(out.has_value, np.uint8).astype(bool),
               "values": [col(out.values[k], np.int64).view(np.float64) if kind in F64_AGGS
                          else col(out.values[k], np.int64) for k, kind in enumerate(self._aggs)]}
        if self._flags & FLAG_KEYED:
            res["key"] = col(out.key, np.uint32)
        return res

    def processWatermarkRaw(self, watermark_ts):
        """processWatermark without building Python objects: returns (n_windows, status)."""
        self._flush()
        out = scotty_windows()
        st = self._check(self._l.scotty_process_watermark(self._h, watermark_ts, ctypes.byref(out)))
        return out.n_windows, st

    # ---- extras
    def droppedCount(self):
        return self._l.scotty_dropped_count(self._h)

    def processedCount(self):
        return self._l.scotty_processed_count(self._h)

    def sliceCount(self):
        return self._l.scotty_slice_count(self._h)

    def firstIndices(self):
        """AGG_FIRST operators: the arrival indices a later window can still return (the FIRST partial of every
        retained non-empty slice, ascending; scotty_first_indices) -- the payloads a shim must keep."""
        self._flush()
        n = self._check(self._l.scotty_first_indices(self._h, None, 0))
        out = np.zeros(max(1, n), dtype=np.int64)
        n = self._check(self._l.scotty_first_indices(self._h, out.ctypes.data, len(out)))
        return out[:n]

    def enableTiming(self, on=True):
        self._check(self._l.scotty_enable_timing(self._h, 1 if on else 0))

    def ingestTiming(self):
        ms, launches, tuples = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._l.scotty_ingest_timing(self._h, ctypes.byref(ms), ctypes.byref(launches),
                                                 ctypes.byref(tuples)))
        return ms.value, launches.value, tuples.value

    def deviceTiming(self):
        """Device milliseconds per class since enableTiming (include/scotty_mi355x.h SCOTTY_TIME_*): a dict
        {ingest, push_other, watermark, result_copy: (ms, intervals)}."""
        out = {}
        for cls, name in enumerate(("ingest", "push_other", "watermark", "result_copy")):
            ms, n = ctypes.c_double(), ctypes.c_uint64()
            self._check(self._l.scotty_device_timing(self._h, cls, ctypes.byref(ms), ctypes.byref(n)))
            out[name] = (ms.value, n.value)
        return out

    def sync(self):
        self._check(self._l.scotty_sync(self._h))

class KeyedSlicingWindowOperator(SlicingWindowOperator):
    """One SlicingWindowOperator per uint32 key, all configured alike -- the per-key HashMap of
    flink-connector/.../KeyedScottyWindowOperator.java:21-86, on the GPU as one keyed engine.

    processElements(keys, ts, values) feeds every key's operator in arrival order; processWatermark(wm)
    returns [(key, AggregateWindow)] of every key's operator (rows of one key contiguous, in the
    reference's order).  KeyedScottyWindowOperator only forwards hasValue() windows (:80): use
    collect(wm) for exactly that stream."""

    _flags = FLAG_KEYED

    def processElement(self, element, ts, key=0):
        self._buf_ts.append(ts)
        self._buf_v.append(element)
        self._buf_k = getattr(self, "_buf_k", [])
        self._buf_k.append(key)

    def _flush(self):
        if self._buf_ts:
            ts, v, k = self._buf_ts, self._buf_v, self._buf_k
            self._buf_ts, self._buf_v, self._buf_k = [], [], []
            self.processElements(k, ts, v)

    def processElements(self, keys, ts, values):
        self._flush()
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        dt = {VALUE_I32: np.int32, VALUE_I64: np.int64, VALUE_F64: np.float64}[self.value_type]
        v = np.ascontiguousarray(values, dtype=dt)
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        assert len(ts) == len(v) == len(k)
        if len(ts):
            self._check(self._l.scotty_process_keyed_elements(self._h, k.ctypes.data, ts.ctypes.data,
                                                              v.ctypes.data, len(ts)))

    def processElementsDevice(self, key_ptr, ts_ptr, val_ptr, n):
        self._flush()
        self._check(self._l.scotty_process_keyed_elements_device(self._h, key_ptr, ts_ptr, val_ptr, n))

    def _windows(self, out):
        n = out.n_windows
        if n == 0:
            return []
        keys = np.ctypeslib.as_array(out.key, shape=(n,)).copy()
        ws = SlicingWindowOperator._windows(self, out)
        return [(int(k), w) for k, w in zip(keys, ws)]

    def collect(self, watermark_ts):
        """What KeyedScottyWindowOperator.processWatermark forwards: hasValue() windows only (:79-82)."""
        return [(k, w) for k, w in self.processWatermark(watermark_ts) if w.hasValue()]

    def keyCount(self):
        return self._l.scotty_key_count(self._h)


class KeyedShardRouter:
    """Host-side keyBy of one keyed stream over G ranks (scotty_route_keyed): key k goes to rank
    keyGroup(k) * G // maxParallelism, keyGroup(k) = murmurHash(k) % maxParallelism -- the SPE's key-group
    assignment that routes tuples to the reference's per-task operators (F/KeyedScottyWindowOperator.java:56-66).
    route() is a stable split: every shard keeps its tuples' arrival order.  Host-only (no GPU needed); rank r then
    feeds route(...)[r] to its own KeyedSlicingWindowOperator, with no collective."""

    def __init__(self, world, max_parallelism=128, threads=0):
        if not 0 < world <= max_parallelism:
            raise ValueError("need 0 < world <= max_parallelism")
        self.world, self.max_parallelism, self.threads = world, max_parallelism, threads
        self._l = lib()

    def shardOf(self, key):
        return int(self._l.scotty_key_shard(key & 0xFFFFFFFF, self.world, self.max_parallelism))

    def route(self, keys, ts, values):
        """-> list of G (keys, ts, values) triples, shard r's tuples in arrival order."""
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        v = np.ascontiguousarray(values)
        if v.dtype not in (np.int32, np.int64, np.float64):
            raise ValueError("values must be int32, int64 or float64")
        n = len(k)
        assert len(t) == n and len(v) == n
        ok, ot, ov = np.empty_like(k), np.empty_like(t), np.empty_like(v)
        off = np.zeros(self.world + 1, dtype=np.uint64)
        rc = self._l.scotty_route_keyed(k.ctypes.data, t.ctypes.data, v.ctypes.data, v.dtype.itemsize, n,
                                        self.world, self.max_parallelism, self.threads, ok.ctypes.data,
                                        ot.ctypes.data, ov.ctypes.data, off.ctypes.data)
        if rc != 0:
            raise ScottyError(rc, "scotty_route_keyed failed")
        o = off.astype(np.int64)
        return [(ok[o[r]:o[r + 1]], ot[o[r]:o[r + 1]], ov[o[r]:o[r + 1]]) for r in range(self.world)]


class ShardedSlicingWindowOperator:
    """One non-keyed stream over the ranks of a torch.distributed group, one GPU each:
    every rank holds the same SlicingWindowOperator and feeds a contiguous arrival chunk of each global
    micro-batch; one all-gather of the per-rank exchange records (RCCL over xGMI for backend "nccl"; host
    staging for "gloo") joins them, and every rank then holds the identical slice store, so processWatermark
    is purely local.  Context-free time windows (the grid path) or count windows (the count path)."""

    def __init__(self, device=0, value_type=VALUE_I32, group=None):
        import torch
        import torch.distributed as dist
        self.dist, self.torch, self.group = dist, torch, group
        self.op = SlicingWindowOperator(device=device, value_type=value_type)
        # sharding count windows by arrival is exact for in-order streams only: the promise lets
        # count-only operators run on the count path, which exports per-rank count cells
        self.op.tune("count_path", 1)
        self.world = dist.get_world_size(group)
        self.dev = torch.device("cuda", device)
        self.staged = dist.get_backend(group) != "nccl"
        # Stream ordering of the RCCL exchange.  With torch imported first, the library's libamdhip64.so.7 is bound
        # to the runtime torch already loaded (same soname), so one HIP runtime serves both: the all-gather is then
        # queued on the op's own stream (a torch.cuda.ExternalStream), between the push and the commit, with no
        # host synchronisation per micro-batch.  When two runtimes are mapped (the library loaded before torch:
        # INTEGRATION.md), a stream of one means nothing to the other, and the exchange falls back to host
        # synchronisation on both sides.  SCOTTY_SHARD_SYNC=1 forces the fallback (A/B).
        self.async_exchange = (not self.staged and _single_hip_runtime()
                               and os.environ.get("SCOTTY_SHARD_SYNC", "0") == "0")
        self._ext = None
        if self.async_exchange:
            self.op.tune("shard_async", 1)
            # the all-gather runs on the op's own stream: push, collective and commit in stream order
            self._ext = torch.cuda.ExternalStream(self.op.opStream(), device=self.dev)
        self._xb = None
        self._assigned = []
        self._measures = set()

    def __getattr__(self, name):  # addWindowFunction, setMaxLateness, processWatermark...
        return getattr(self.op, name)

    def addWindowAssigner(self, window):
        self.op.addWindowAssigner(window)
        self._assigned.append(window)
        self._measures.add(window.measure)  # kept incrementally: per-chunk checks must not walk 1000 windows

    def _count_and_time(self):
        return {0, 1} <= self._measures  # SCOTTY_MEASURE_TIME, SCOTTY_MEASURE_COUNT

    def _bufs(self):
        if self._xb is None:
            words = self.op.shardXBytes() // 8
            t = self.torch
            self._xb = t.empty(words, dtype=t.int64, device=self.dev)
            self._gb = t.empty(words * self.world, dtype=t.int64, device=self.dev)
            if self.staged:
                self._hx = t.empty(words, dtype=t.int64)
                self._hg = t.empty(words * self.world, dtype=t.int64)
        return self._xb, self._gb

    def processChunk(self, ts_ptr, val_ptr, n, ts0=0, n_before=None, n_total=None, ts_before=None, ts_last=None):
        """This rank's arrival chunk of the next global micro-batch (device pointers); ts0 = the global first
        tuple's timestamp (read on the very first batch only).  n_before / n_total: tuples of the lower ranks /
        of all ranks in this micro-batch (count windows number tuples globally); ts_before / ts_last: the largest
        timestamp on the lower ranks / in the whole micro-batch (count + time windows); gathered when not given."""
        timed = self._count_and_time()
        counted = 1 in self._measures  # SCOTTY_MEASURE_COUNT
        if not counted:  # time windows only (the grid path): no count offsets, no extra collective
            xb, gb = self._bufs()
            self.op.shardPush(ts_ptr, val_ptr, n, ts0, xb.data_ptr())
            self._exchange(xb, gb)
            return
        if n_before is None or n_total is None or (timed and (ts_before is None or ts_last is None)):
            # one small all-gather of {n, first ts, last ts} per rank (count windows number tuples globally; time
            # windows on the count path decide a chunk's edges from the max ts before it, CEngine::time_edges)
            t = self.torch
            first, last = self.op.shardBounds(ts_ptr, n) if timed else (0, 0)
            mine = t.tensor([n, first, last], dtype=t.int64, device=self.dev if not self.staged else "cpu")
            allv = t.empty(3 * self.world, dtype=t.int64, device=mine.device)
            self.dist.all_gather_into_tensor(allv, mine, group=self.group)
            g = allv.view(self.world, 3).tolist()  # .tolist() waits for the collective on torch's stream
            r = self.dist.get_rank(self.group)
            n_before, n_total = int(sum(x[0] for x in g[:r])), int(sum(x[0] for x in g))
            lasts = [x[2] for x in g if x[0] > 0]
            ts_before = max([x[2] for x in g[:r] if x[0] > 0], default=-2**63)
            ts_last = max(lasts, default=-2**63)
        xb, gb = self._bufs()
        if timed:
            self.op.shardPushTimed(ts_ptr, val_ptr, n, ts0, n_before, n_total, ts_before, ts_last, xb.data_ptr())
        else:
            self.op.shardPushCounted(ts_ptr, val_ptr, n, ts0, n_before, n_total, xb.data_ptr())
        self._exchange(xb, gb)

    def _exchange(self, xb, gb):
        """All-gather of the ranks' exchange records (RCCL for "nccl", host-staged for "gloo"), then the commit."""
        if self.staged:
            self._hx.copy_(xb)
            self.dist.all_gather_into_tensor(self._hg, self._hx, group=self.group)
            gb.copy_(self._hg)
            self.torch.cuda.synchronize(self.dev)
        elif self.async_exchange:
            with self.torch.cuda.stream(self._ext):  # behind the push, ahead of the commit, on the op's stream
                self.dist.all_gather_into_tensor(gb, xb, group=self.group)
            self.op.shardCommit(gb.data_ptr(), self.world)
            # torch's stream waits for the chunk's push and commit (one event, no host wait): the caller's input
            # tensors may be freed and their memory reused by torch as soon as processChunk returns, and torch's
            # allocator only orders reuse on its own streams
            self.op.streamOrder(self.torch.cuda.current_stream(self.dev).cuda_stream, False)
            return
        else:
            # the record is complete: the push synchronised the library's stream before returning
            self.dist.all_gather_into_tensor(gb, xb, group=self.group)
            self.torch.cuda.current_stream(self.dev).synchronize()  # the gathered records have landed
        self.op.shardCommit(gb.data_ptr(), self.world)


from . import workloads  # noqa: E402,F401
