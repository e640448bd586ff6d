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


# SUM_F64 contract (north_star "within 1e-6 relative", stated for signed streams): the product reassociates the
# reference's arrival-order left fold (AggregateValueState.addElement / merge, S/state/AggregateValueState.java:23-31,
# 55-69: per-cell atomicAdd(double), then slices, then windows), and two summation orders of the same n terms differ by
# at most 2(n-1)u * sum|x| (u = 2^-53).  So every window's f64 sum is checked against |got - ref| <= F64_REL * S with
# S = sum of |x| over the window's tuples (the same window's SUM_F64 over |x|, from an abs-valued twin operator): a
# bound that holds for cancelling windows, where a plain relative bound on |ref| cannot hold for any reassociation.
F64_REL = 1e-6


def f64_close(p, q, scale):
    """|p - q| <= F64_REL * scale (scale = sum |x| of the window), NaN only with NaN."""
    if isinstance(q, float) and math.isnan(q):
        return isinstance(p, float) and math.isnan(p)
    return abs(p - q) <= F64_REL * scale


def same_windows(a, b, f64_cols=(), scale=None):
    """Window lists equal position by position: start, end, measure, hasValue bit-exact; values bit-exact
    except the columns in f64_cols (SUM_F64), compared by f64_close against scale[i][j] = sum |x| of window i
    (``scale`` None: the lists come from the same order of the same stream, compared within F64_REL * |q|)."""
    assert len(a) == len(b), ("window count", len(a), len(b))
    for i, (x, y) in enumerate(zip(a, b)):
        assert (x.getStart(), x.getEnd(), x.getMeasure(), x.hasValue()) == \
               (y.getStart(), y.getEnd(), y.getMeasure(), y.hasValue()), (i, x, y)
        xv, yv = x.getAggValues(), y.getAggValues()
        assert len(xv) == len(yv), (i, x, y)
        for j, (p, q) in enumerate(zip(xv, yv)):
            if j in f64_cols:
                sc = abs(q) if scale is None else scale[i][j]
                assert f64_close(p, q, sc), (i, j, p, q, sc)
            else:
                assert p == q, (i, j, p, q, x, y)


def abs_twin(cfg):
    """An oracle operator with cfg's windows / functions / lateness, fed |x|: its SUM_F64 columns are the sum |x|
    scale of every window of the checked operator (same timestamps, so the same windows in the same order)."""
    from oracle.oracle import OracleOperator
    ora = OracleOperator()
    for a in cfg["aggs"]:
        ora.addWindowFunction(a)
    if cfg.get("lateness") is not None:
        ora.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        ora.addWindowAssigner(w)
    return ora


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
    ora.cfg = cfg  # run_schedule builds the f64 scale twin from it
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
    twin = abs_twin(ora.cfg) if value_type == "f64" and f64_cols and hasattr(ora, "cfg") else None
    for step in schedule:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi <= lo:
                continue
            gpu.processElements(ts[lo:hi], vals[lo:hi])
            if value_type == "f64":
                fails += ora.processElements(ts[lo:hi], np.zeros(hi - lo, dtype=np.int64), vals[lo:hi])
                if twin is not None:
                    twin.processElements(ts[lo:hi], np.zeros(hi - lo, dtype=np.int64), np.abs(vals[lo:hi]))
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
                if twin is not None:
                    with pytest.raises(JavaError):
                        twin.processWatermark(step[1])
                continue
            b = ora.processWatermark(step[1])
            scale = None
            if twin is not None:
                tw = twin.processWatermark(step[1])
                assert len(tw) == len(b)
                scale = [w.getAggValues() if w.hasValue() else [0.0] * len(f64_cols) for w in tw]
            same_windows(a, b, f64_cols=f64_cols, scale=scale)
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

    def processElements(self, keys, ts, vals, absolute=False):
        import numpy as np
        keys = np.asarray(keys)
        if absolute:  # the f64 scale twin (see abs_twin)
            vals = np.abs(vals)
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


def same_keyed_arrays(got, exp, f64_cols=(), scale=None):
    """Two keyed processWatermarkArrays results: the same rows key by key (keys as a set, each key's rows in order,
    as same_keyed_windows), compared column-wise in numpy; f64 columns in f64_cols by f64_close, against
    ``scale`` = the processWatermarkArrays result of an |x|-fed twin of ``exp``'s operator (sum |x| per row)."""
    import numpy as np
    n = len(exp["start"])
    assert len(got["start"]) == n
    if n == 0:
        return 0
    og, oe = np.argsort(got["key"], kind="stable"), np.argsort(exp["key"], kind="stable")
    for c in ("key", "start", "end", "measure", "has_value"):
        assert np.array_equal(got[c][og], exp[c][oe]), c
    hv = exp["has_value"][oe]
    if scale is not None:  # the twin's rows, key by key in the same order
        os_ = np.argsort(scale["key"], kind="stable")
        for c in ("key", "start", "end"):
            assert np.array_equal(scale[c][os_], exp[c][oe]), ("scale twin", c)
    for i, (a, b) in enumerate(zip(got["values"], exp["values"])):
        a, b = a[og][hv], b[oe][hv]
        if i in f64_cols:
            nan = np.isnan(b)
            assert np.array_equal(np.isnan(a), nan), i
            sc = np.abs(b) if scale is None else scale["values"][i][os_][hv]
            assert np.all(np.abs(a[~nan] - b[~nan]) <= F64_REL * sc[~nan]), i
        else:
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), i
    return n


def same_keyed_windows(rows, expected, f64_cols=(), scale=None):
    """rows: [(key, AggregateWindow)] of the product; expected: {key: [AggregateWindow]} of the oracle.
    Keys compare as a set (Java HashMap order is not a contract); windows of one key position by position.
    scale: {key: [AggregateWindow]} of the |x|-fed twin (KeyedOracle.processElements(..., absolute=True))."""
    got = {}
    for k, w in rows:
        got.setdefault(k, []).append(w)
    exp = {k: v for k, v in expected.items() if v}
    assert set(got) == set(exp), ("keys", sorted(set(got) ^ set(exp))[:10])
    for k in exp:
        sc = None
        if scale is not None and f64_cols:
            sc = [w.getAggValues() if w.hasValue() else [0.0] * 8 for w in scale[k]]
        same_windows(got[k], exp[k], f64_cols=f64_cols, scale=sc)
    return sum(len(v) for v in exp.values())
