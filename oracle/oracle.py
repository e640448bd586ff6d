"""ctypes wrapper of the CPU ORACLE (oracle/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  It mirrors the reference operator's method names
(S/SlicingWindowOperator.java:21-69) so the transcribed JUnit tests read like
the reference's own.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")

WIN_TUMBLING, WIN_SLIDING, WIN_SESSION, WIN_FIXED_BAND = 0, 1, 2, 3
WIN_TEST_SCRIPTED, WIN_TEST_NULLCTX = 100, 101
TIME, COUNT = 0, 1
AGG_SUM_I32, AGG_COUNT, AGG_MIN_I32, AGG_MAX_I32 = 0, 1, 2, 3
AGG_SUM_I64, AGG_MIN_I64, AGG_MAX_I64 = 4, 5, 6
AGG_SUM_F64, AGG_MIN_F64, AGG_MAX_F64 = 7, 8, 9
AGG_FIRST = 10  # arrival index of the first partial's tuple (ORC_AGG_FIRST)
AGG_SUB_I32 = 100
AGG_INVERTIBLE = 0x10000
STATE_MEMORY, STATE_MOCK = 0, 1
F64_AGGS = (AGG_SUM_F64, AGG_MIN_F64, AGG_MAX_F64)

ERR_NAMES = {-1: "IndexOutOfBoundsException", -2: "NullPointerException",
             -3: "NoSuchElementException", -4: "ArithmeticException", -5: "IllegalArgument",
             -6: "ReferenceWouldHang"}
ERR_HANG = -6


class JavaError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class SliceInfo(ctypes.Structure):
    _fields_ = [("t_start", ctypes.c_int64), ("t_end", ctypes.c_int64), ("t_first", ctypes.c_int64),
                ("t_last", ctypes.c_int64), ("c_start", ctypes.c_int64), ("c_last", ctypes.c_int64),
                ("type_fixed", ctypes.c_int32), ("flex_count", ctypes.c_int32),
                ("is_lazy", ctypes.c_int32), ("n_records", ctypes.c_int32)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64, i32, dbl = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        sig = {
            "orc_create": (P, [ctypes.c_int]),
            "orc_destroy": (None, [P]),
            "orc_last_error": (ctypes.c_char_p, [P]),
            "orc_set_mod_order": (None, [P, ctypes.c_int, ctypes.c_uint64]),
            "orc_add_window": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, i64, i64]),
            "orc_add_aggregation": (ctypes.c_int, [P, ctypes.c_int]),
            "orc_set_max_lateness": (ctypes.c_int, [P, i64]),
            "orc_process_element": (ctypes.c_int, [P, i64, dbl, i64]),
            "orc_process_elements": (ctypes.c_int, [P, P, P, P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
            "orc_process_watermark": (ctypes.c_int, [P, i64]),
            "orc_num_windows": (i64, [P]),
            "orc_window": (ctypes.c_int, [P, i64, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i32),
                                          ctypes.POINTER(i32), ctypes.POINTER(i32)]),
            "orc_window_value": (ctypes.c_int, [P, i64, i32, ctypes.POINTER(i64), ctypes.POINTER(dbl),
                                                ctypes.POINTER(i32)]),
            "orc_store_size": (ctypes.c_int, [P]),
            "orc_slice": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(SliceInfo)]),
            "orc_slice_records": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(i64), ctypes.c_int]),
            "orc_slice_value": (ctypes.c_int, [P, ctypes.c_int, i32, ctypes.POINTER(i64), ctypes.POINTER(dbl),
                                               ctypes.POINTER(i32)]),
            "orc_slice_num_values": (ctypes.c_int, [P, ctypes.c_int]),
            "orc_store_append_new_slice": (ctypes.c_int, [P, i64, i64, ctypes.c_int, ctypes.c_int]),
            "orc_factory_would_be_lazy": (ctypes.c_int, [P]),
            "orc_manager_process_element": (ctypes.c_int, [P, i64, i64]),
            "orc_store_find_slice_index_by_ts": (ctypes.c_int, [P, i64]),
            "orc_store_insert_value_to_slice": (ctypes.c_int, [P, ctypes.c_int, i64, i64]),
            "orc_store_insert_value_to_current": (ctypes.c_int, [P, i64, i64]),
            "orc_manager_flags": (ctypes.c_int, [P]),
            "orc_max_lateness": (i64, [P]),
            "orc_current_count": (i64, [P]),
            "orc_keyed_create": (P, [ctypes.c_int]),
            "orc_keyed_destroy": (None, [P]),
            "orc_keyed_add_window": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, i64, i64]),
            "orc_keyed_add_aggregation": (ctypes.c_int, [P, ctypes.c_int]),
            "orc_keyed_set_max_lateness": (ctypes.c_int, [P, i64]),
            "orc_keyed_num_keys": (i64, [P]),
            "orc_keyed_process": (i64, [P, P, P, P, P, i64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class Window:
    """An emitted window (C/AggregateWindow.java:8-21)."""

    def __init__(self, start, end, measure, has_value, values):
        self.start, self.end, self.measure = start, end, measure
        self._has_value, self._values = has_value, values

    def getStart(self):
        return self.start

    def getEnd(self):
        return self.end

    def getMeasure(self):
        return self.measure

    def hasValue(self):
        return self._has_value

    def getAggValues(self):
        return list(self._values)

    def key(self):
        return (self.start, self.end, self.measure, self._has_value, tuple(self._values))

    def __repr__(self):
        return "Window(%d,%d,m=%d,%s)" % (self.start, self.end, self.measure, self._values)


class OracleOperator:
    """SlicingWindowOperator restated on the CPU (S/SlicingWindowOperator.java:21-69)."""

    def __init__(self, state_mode=STATE_MEMORY):
        self._l = lib()
        self._h = self._l.orc_create(state_mode)
        self._aggs = []

    def __del__(self):
        try:
            if self._h:
                self._l.orc_destroy(self._h)
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise JavaError(rc, self._l.orc_last_error(self._h).decode())
        return rc

    # --- reference API names
    def addWindowAssigner(self, kind, measure=None, a=0, b=0):
        if measure is None:  # a window-spec object (kind, measure, a, b)
            kind, measure, a, b = kind.kind, kind.measure, kind.a, kind.b
        self._check(self._l.orc_add_window(self._h, kind, measure, a, b))

    def addWindowFunction(self, kind):
        self._aggs.append(kind & 0xFFFF)
        return self._check(self._l.orc_add_aggregation(self._h, kind))

    addAggregation = addWindowFunction

    def setMaxLateness(self, l):
        self._check(self._l.orc_set_max_lateness(self._h, l))

    def setModOrder(self, mode, seed=0):
        self._l.orc_set_mod_order(self._h, mode, seed)

    def processElement(self, value, ts):
        self._check(self._l.orc_process_element(self._h, int(value), float(value), ts))

    def processElements(self, ts, values, values_f=None):
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vi = np.ascontiguousarray(values, dtype=np.int64)
        vf = None if values_f is None else np.ascontiguousarray(values_f, dtype=np.float64)
        nf = ctypes.c_size_t(0)
        self._l.orc_process_elements(self._h, ts.ctypes.data, vi.ctypes.data,
                                     None if vf is None else vf.ctypes.data, len(ts), ctypes.byref(nf))
        return nf.value

    def processWatermark(self, wm):
        self._check(self._l.orc_process_watermark(self._h, wm))
        return self.results()

    def results(self):
        out = []
        n = self._l.orc_num_windows(self._h)
        s, e = ctypes.c_int64(), ctypes.c_int64()
        m, hv, nv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        vi, vf, isn = ctypes.c_int64(), ctypes.c_double(), ctypes.c_int32()
        for i in range(n):
            self._l.orc_window(self._h, i, ctypes.byref(s), ctypes.byref(e), ctypes.byref(m), ctypes.byref(hv),
                               ctypes.byref(nv))
            vals = []
            present = [k for k in range(len(self._aggs))]
            for j in range(nv.value):
                self._l.orc_window_value(self._h, i, j, ctypes.byref(vi), ctypes.byref(vf), ctypes.byref(isn))
                kind = self._aggs[present[j]] if j < len(present) else 0
                if isn.value:
                    vals.append(None)
                else:
                    vals.append(vf.value if kind in F64_AGGS else vi.value)
            out.append(Window(s.value, e.value, m.value, bool(hv.value), vals))
        return out

    # --- component hooks (SliceManagerTest / SliceFactoryTest / LazyAggregateStoreTest)
    def store_size(self):
        return self._l.orc_store_size(self._h)

    def slice(self, i):
        info = SliceInfo()
        self._check(self._l.orc_slice(self._h, i, ctypes.byref(info)))
        return info

    def slice_records(self, i):
        buf = (ctypes.c_int64 * 4096)()
        n = self._check(self._l.orc_slice_records(self._h, i, buf, 4096))
        return [buf[k] for k in range(n)]

    def slice_values(self, i):
        n = self._check(self._l.orc_slice_num_values(self._h, i))
        vi, vf, isn = ctypes.c_int64(), ctypes.c_double(), ctypes.c_int32()
        out = []
        for j in range(n):
            self._l.orc_slice_value(self._h, i, j, ctypes.byref(vi), ctypes.byref(vf), ctypes.byref(isn))
            out.append(None if isn.value else vi.value)
        return out

    def store_append_new_slice(self, start, end, fixed=False, flex_count=1):
        self._check(self._l.orc_store_append_new_slice(self._h, start, end, 1 if fixed else 0, flex_count))

    def factory_would_be_lazy(self):
        return bool(self._l.orc_factory_would_be_lazy(self._h))

    def manager_process_element(self, value, ts):
        self._check(self._l.orc_manager_process_element(self._h, value, ts))

    def find_slice_index_by_ts(self, ts):
        return self._l.orc_store_find_slice_index_by_ts(self._h, ts)

    def insert_value_to_slice(self, idx, value, ts):
        self._check(self._l.orc_store_insert_value_to_slice(self._h, idx, value, ts))

    def insert_value_to_current(self, value, ts):
        self._check(self._l.orc_store_insert_value_to_current(self._h, value, ts))

    def flags(self):
        f = self._l.orc_manager_flags(self._h)
        return {"hasContextAwareWindow": bool(f & 1), "isSessionWindowCase": bool(f & 2),
                "hasCountMeasure": bool(f & 4), "hasFixedWindows": bool(f & 8), "hasTimeMeasure": bool(f & 16)}

    def max_lateness(self):
        return self._l.orc_max_lateness(self._h)


class KeyedOracleThreads:
    """KeyedScottyWindowOperator (flink-connector/.../KeyedScottyWindowOperator.java:41-86) restated on the CPU with
    the key space split over T threads (partition = key % T, as an upstream keyBy of parallelism T delivers).
    CPU baseline of the keyed configuration; process() returns the forwarded (hasValue) window count."""

    def __init__(self, threads):
        self._l = lib()
        self.threads = int(threads)
        self._h = self._l.orc_keyed_create(self.threads)

    def __del__(self):
        try:
            if self._h:
                self._l.orc_keyed_destroy(self._h)
        except Exception:
            pass

    def addWindowAssigner(self, kind, measure, a=0, b=0):
        self._l.orc_keyed_add_window(self._h, kind, measure, a, b)

    def addWindowFunction(self, kind):
        self._l.orc_keyed_add_aggregation(self._h, kind)

    def setMaxLateness(self, l):
        self._l.orc_keyed_set_max_lateness(self._h, l)

    def partition(self, keys, ts, values):
        """Rows grouped by partition (stable: arrival order kept inside each partition) + offsets."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        part = (keys % self.threads).astype(np.uint8)
        order = np.argsort(part, kind="stable")
        off = np.zeros(self.threads + 1, dtype=np.int64)
        off[1:] = np.cumsum(np.bincount(part, minlength=self.threads))
        return (off, np.ascontiguousarray(keys[order]), np.ascontiguousarray(np.asarray(ts, dtype=np.int64)[order]),
                np.ascontiguousarray(np.asarray(values, dtype=np.int64)[order]))

    def process(self, parted, watermark):
        off, k, t, v = parted
        n = self._l.orc_keyed_process(self._h, off.ctypes.data, k.ctypes.data, t.ctypes.data, v.ctypes.data,
                                      int(watermark))
        if n < 0:
            raise JavaError(n, "keyed oracle error %d" % n)
        return n

    def numKeys(self):
        return self._l.orc_keyed_num_keys(self._h)
