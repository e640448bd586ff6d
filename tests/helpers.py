"""Shared helpers for the parity tests (oracle = CPU checker, product = MI355X C-ABI)."""
import importlib
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def product():
    return importlib.import_module("scotty-window-processor_amd")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def same_windows(a, b, f64_cols=(), rel=1e-6):
    """Window lists equal position by position: start, end, measure, hasValue bit-exact; values bit-exact
    except the columns in f64_cols, compared within ``rel`` relative tolerance (SUM_F64, north_star)."""
    assert len(a) == len(b), ("window count", len(a), len(b))
    for i, (x, y) in enumerate(zip(a, b)):
        assert (x.getStart(), x.getEnd(), x.getMeasure(), x.hasValue()) == \
               (y.getStart(), y.getEnd(), y.getMeasure(), y.hasValue()), (i, x, y)
        xv, yv = x.getAggValues(), y.getAggValues()
        assert len(xv) == len(yv), (i, x, y)
        for j, (p, q) in enumerate(zip(xv, yv)):
            if j in f64_cols:
                if isinstance(p, float) and math.isnan(p):
                    assert isinstance(q, float) and math.isnan(q), (i, j, p, q)
                else:
                    assert abs(p - q) <= rel * max(1.0, abs(q)), (i, j, p, q)
            else:
                assert p == q, (i, j, p, q, x, y)


def build_ops(cfg, value_type="i32", device=0, tune=None):
    """Create (product, oracle) operators with the same windows / functions / lateness.
    cfg: dict(windows=[spec...], aggs=[kind...], lateness=int|None); tune: scotty_tune knobs of the product."""
    from oracle.oracle import OracleOperator
    pkg = product()
    vt = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[value_type]
    gpu = pkg.SlicingWindowOperator(device=device, value_type=vt)
    for k, v in (tune or {}).items():
        gpu.tune(k, v)
    ora = OracleOperator()
    for op in (gpu, ora):
        for a in cfg["aggs"]:
            op.addWindowFunction(a)
        if cfg.get("lateness") is not None:
            op.setMaxLateness(cfg["lateness"])
        for w in cfg["windows"]:
            op.addWindowAssigner(w)
    return gpu, ora


def run_schedule(gpu, ora, ts, vals, schedule, value_type="i32", f64_cols=()):
    """schedule: list of ("push", lo, hi) / ("wm", watermark).  Compares every watermark's windows and the
    number of too-late tuples (product drops + counts them; the reference throws per tuple)."""
    import numpy as np
    n_windows = 0
    fails = 0
    for step in schedule:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi <= lo:
                continue
            gpu.processElements(ts[lo:hi], vals[lo:hi])
            if value_type == "f64":
                fails += ora.processElements(ts[lo:hi], np.zeros(hi - lo, dtype=np.int64), vals[lo:hi])
            else:
                fails += ora.processElements(ts[lo:hi], vals[lo:hi])
        else:
            try:
                a = gpu.processWatermark(step[1])
            except product().ScottyError as e:
                if e.code != -5:
                    raise
                # the reference throws IndexOutOfBoundsException in processWatermark (e.g. a count trigger with
                # the watermark before the oldest slice, S/WindowManager.java:109-112): the oracle must as well,
                # and both keep their state (the exception precedes every update)
                import pytest
                from oracle.oracle import JavaError
                with pytest.raises(JavaError):
                    ora.processWatermark(step[1])
                continue
            b = ora.processWatermark(step[1])
            same_windows(a, b, f64_cols=f64_cols)
            n_windows += len(a)
            assert gpu.droppedCount() == fails, ("dropped", gpu.droppedCount(), fails)
    return n_windows


def interval_schedule(ts, n_intervals, lag, pushes_per_interval=1):
    """Cut the arrival sequence into n_intervals equal intervals; after each, a watermark max_ts - lag."""
    import numpy as np
    n = len(ts)
    sched = []
    bounds = np.linspace(0, n, n_intervals + 1).astype(np.int64)
    for i in range(n_intervals):
        lo, hi = int(bounds[i]), int(bounds[i + 1])
        sub = np.linspace(lo, hi, pushes_per_interval + 1).astype(np.int64)
        for j in range(pushes_per_interval):
            sched.append(("push", int(sub[j]), int(sub[j + 1])))
        if hi > 0:
            sched.append(("wm", int(ts[:hi].max()) - lag))
    return sched


class KeyedOracle:
    """One OracleOperator per key, created on the key's first tuple with the same windows / functions /
    lateness -- the HashMap of flink-connector/.../KeyedScottyWindowOperator.java:21-66.  Test checker."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.ops = {}      # key -> OracleOperator, insertion order = creation order
        self.failed = 0

    def _new(self):
        from oracle.oracle import OracleOperator
        op = OracleOperator()
        for a in self.cfg["aggs"]:
            op.addWindowFunction(a)
        if self.cfg.get("lateness") is not None:
            op.setMaxLateness(self.cfg["lateness"])
        for w in self.cfg["windows"]:
            op.addWindowAssigner(w)
        return op

    def processElements(self, keys, ts, vals):
        import numpy as np
        keys = np.asarray(keys)
        for k in keys:  # creation order = first appearance
            k = int(k)
            if k not in self.ops:
                self.ops[k] = self._new()
        order = np.argsort(keys, kind="stable")
        ks = keys[order]
        bounds = np.flatnonzero(np.diff(ks)) + 1
        for seg in np.split(np.arange(len(ks)), bounds):
            if len(seg) == 0:
                continue
            idx = order[seg]
            op = self.ops[int(ks[seg[0]])]
            if vals.dtype.kind == "f":
                self.failed += op.processElements(ts[idx], np.zeros(len(idx), dtype=np.int64), vals[idx])
            else:
                self.failed += op.processElements(ts[idx], vals[idx])

    def processWatermark(self, wm):
        # KeyedScottyWindowOperator.processWatermark loops over every key's operator (:77); an exception of
        # one key's processWatermark propagates out of the loop
        return {k: op.processWatermark(wm) for k, op in self.ops.items()}


def same_keyed_arrays(got, exp, f64_cols=()):
    """Two keyed processWatermarkArrays results: the same rows key by key (keys as a set, each key's rows in order,
    as same_keyed_windows), compared column-wise in numpy; f64 columns in f64_cols within 1e-6 relative."""
    import numpy as np
    n = len(exp["start"])
    assert len(got["start"]) == n
    if n == 0:
        return 0
    og, oe = np.argsort(got["key"], kind="stable"), np.argsort(exp["key"], kind="stable")
    for c in ("key", "start", "end", "measure", "has_value"):
        assert np.array_equal(got[c][og], exp[c][oe]), c
    hv = exp["has_value"][oe]
    for i, (a, b) in enumerate(zip(got["values"], exp["values"])):
        a, b = a[og][hv], b[oe][hv]
        if i in f64_cols:
            nan = np.isnan(b)
            assert np.array_equal(np.isnan(a), nan), i
            assert np.all(np.abs(a[~nan] - b[~nan]) <= 1e-6 * np.maximum(1.0, np.abs(b[~nan]))), i
        else:
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), i
    return n


def same_keyed_windows(rows, expected, f64_cols=()):
    """rows: [(key, AggregateWindow)] of the product; expected: {key: [AggregateWindow]} of the oracle.
    Keys compare as a set (Java HashMap order is not a contract); windows of one key position by position."""
    got = {}
    for k, w in rows:
        got.setdefault(k, []).append(w)
    exp = {k: v for k, v in expected.items() if v}
    assert set(got) == set(exp), ("keys", sorted(set(got) ^ set(exp))[:10])
    for k in exp:
        same_windows(got[k], exp[k], f64_cols=f64_cols)
    return sum(len(v) for v in exp.values())
