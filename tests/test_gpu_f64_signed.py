"""SUM_F64 on signed, cancelling streams at the bench's batch size (2^26 tuples per micro-batch), on all three engines:
the grid path (1000 tumbling windows), the exact engine (session + sliding windows, non-keyed) and the keyed engine
(2^20 keys, tumbling + sliding).

The contract (tests/helpers.py F64_REL): the reference folds each window's values left to right in arrival order
(AggregateValueState.addElement / merge, S/state/AggregateValueState.java:23-31, 55-69); the product reassociates
that fold (per-cell atomicAdd(double), slices, windows).  Any two summation orders of the same n doubles differ by at
most 2(n-1)u * sum|x| (u = 2^-53), so the bound that holds -- and that these tests check -- is

    |got - ref| <= 1e-6 * sum|x| over the window's tuples,

not 1e-6 * |ref|, which no reassociation can promise when the window's sum cancels to near zero.  Each window is
checked against its exactly rounded sum (numpy long double prefix sums; the arrival-order fold the reference computes
is within n * u * sum|x| of it, 1e-8 * sum|x| at n = 2^26, so the check uses 0.99e-6) and COUNT bit-exactly.  The worst
error seen is reported in units of sum|x| and of |sum|, the latter to show the windows really cancel."""
import numpy as np
import pytest

from helpers import product, F64_REL

pytestmark = pytest.mark.gpu

N = 1 << 26
BOUND = 0.99 * F64_REL  # room for the reference's own arrival-order rounding (<= n u sum|x|)


def _not_pow2(x):
    return x + 1 if x & (x - 1) == 0 else x


def _signed(rng, n):
    # mixed signs, magnitudes over 6 decades: window sums cancel to far below their sum |x|
    return rng.standard_normal(n) * np.exp(rng.uniform(-7, 7, n))


def _check(rows, lo, hi, pre, pabs):
    """rows: (start, end, has, sum, count) arrays; lo/hi tuple ranges of each row in the sorted order."""
    s, has, got, cnt = rows
    if not np.any(has):
        assert np.all(hi - lo == 0)
        return 0, 0.0, 0.0
    exp = pre[hi] - pre[lo]
    sabs = pabs[hi] - pabs[lo]
    assert np.array_equal(cnt[has], (hi - lo)[has])
    assert np.all((hi - lo)[~has] == 0)
    err = np.abs(got[has].astype(np.longdouble) - exp[has])
    assert np.all(err <= BOUND * sabs[has]), float(np.max(err / np.maximum(sabs[has], 1e-300)))
    worst_abs = float(np.max(err / np.maximum(sabs[has], 1e-300)))
    with np.errstate(divide="ignore", invalid="ignore"):
        worst_rel = float(np.nanmax(err / np.abs(exp[has])))
    return int(has.sum()), worst_abs, worst_rel


def _arrays_rows(arrs):
    return arrs["start"], arrs["has_value"], arrs["values"][0], arrs["values"][1]


def test_f64_signed_grid_path_bench_scale():
    """Grid path: 1000 in-order tumbling windows of 50-1000 ms, two micro-batches of 2^26 tuples."""
    import torch
    pkg = product()
    dev = torch.device("cuda", 0)
    rate = N // 1000
    sizes = [_not_pow2(50 + (x % 951)) for x in pkg.workloads.random_tumbling_sizes()]
    op = pkg.SlicingWindowOperator(device=0, value_type=pkg.VALUE_F64)
    op.addWindowFunction(pkg.AGG_SUM_F64)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for s in sizes:
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    assert op._debug_stat(5) in (-1, 0, 1)
    rng = np.random.default_rng(61)
    vals, ts_all, got = [], [], []
    for step in range(2):
        ts = np.arange(N, dtype=np.int64) // rate + step * 1000
        v = _signed(rng, N)
        dts, dv = torch.from_numpy(ts).to(dev), torch.from_numpy(v).to(dev)
        torch.cuda.synchronize(dev)
        op.processElementsDevice(dts.data_ptr(), dv.data_ptr(), N)
        assert op._debug_stat(5) == 1  # the grid path
        got.append(op.processWatermarkArrays(step * 1000 + 999))
        vals.append(v)
        ts_all.append(ts)
        del dts, dv
    v = np.concatenate(vals)
    ts = np.concatenate(ts_all)
    pre = np.concatenate([[0], np.cumsum(v.astype(np.longdouble))])
    pabs = np.concatenate([[0], np.cumsum(np.abs(v).astype(np.longdouble))])
    checked = 0
    for a in got:
        lo = np.searchsorted(ts, a["start"], side="left")
        hi = np.searchsorted(ts, a["end"], side="left")
        n, wa, wr = _check(_arrays_rows(a), lo, hi, pre, pabs)
        checked += n
    assert checked > 1000
    print("grid: %d windows, worst |err|/sum|x| %.2e, worst |err|/|sum| %.2e" % (checked, wa, wr))


def test_f64_signed_exact_engine_bench_scale():
    """Exact engine (non-keyed, SessionWindow(gap 50) + SlidingWindow(500, 100)): in-order stream of 2 x 2^26 tuples
    with silences that close sessions, so session and sliding windows both emit.  A window holds the slices it contains
    by tLast (S/state/AggregateWindowState.java:25-31): with the window size a multiple of the slide every window ends
    on a slice edge, and a session window [start, last + gap) ends before the next session's first slice, so each
    window's tuples are the in-order stream's range [start, end)."""
    import torch
    pkg = product()
    dev = torch.device("cuda", 0)
    rate = N // 1000
    op = pkg.SlicingWindowOperator(device=0, value_type=pkg.VALUE_F64)
    op.addWindowFunction(pkg.AGG_SUM_F64)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.SessionWindow(pkg.WindowMeasure.Time, 50))
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 500, 100))
    rng = np.random.default_rng(62)
    vals, ts_all, got = [], [], []
    for step in range(2):
        idx = np.arange(N, dtype=np.int64)
        ts = idx // rate + step * 1300 + (idx >= N // 2) * 100  # a 100 ms silence mid batch: a session closes
        v = _signed(rng, N)
        dts, dv = torch.from_numpy(ts).to(dev), torch.from_numpy(v).to(dev)
        torch.cuda.synchronize(dev)
        op.processElementsDevice(dts.data_ptr(), dv.data_ptr(), N)
        assert op._debug_stat(5) == 2  # the exact engine
        got.append(op.processWatermarkArrays(int(ts[-1])))
        vals.append(v)
        ts_all.append(ts)
        del dts, dv
    v = np.concatenate(vals)
    ts = np.concatenate(ts_all)
    assert np.all(np.diff(ts) >= 0)
    pre = np.concatenate([[0], np.cumsum(v.astype(np.longdouble))])
    pabs = np.concatenate([[0], np.cumsum(np.abs(v).astype(np.longdouble))])
    checked = sessions = 0
    for a in got:
        lo = np.searchsorted(ts, a["start"], side="left")
        hi = np.searchsorted(ts, a["end"], side="left")
        n, wa, wr = _check(_arrays_rows(a), lo, hi, pre, pabs)
        checked += n
        sessions += int(np.count_nonzero(a["end"] - a["start"] != 500))
    assert checked > 20 and sessions >= 2
    print("exact: %d windows (%d sessions), worst |err|/sum|x| %.2e, worst |err|/|sum| %.2e"
          % (checked, sessions, wa, wr))


def test_f64_signed_keyed_engine_bench_scale():
    """Keyed engine: 2^20 uniform keys, TumblingWindow(1000) + SlidingWindow(2001, 1000), two in-order micro-batches
    of 2^26 tuples (the sort-free path from the second batch on, the replay of new keys in the first).  Expected
    per (key, window) from the tuples sorted by (key, ts) -- stable, so each key keeps its arrival order."""
    import torch
    pkg = product()
    dev = torch.device("cuda", 0)
    rate = N // 1000
    nkeys = 1 << 20
    op = pkg.KeyedSlicingWindowOperator(device=0, value_type=pkg.VALUE_F64)
    op.addWindowFunction(pkg.AGG_SUM_F64)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, 1000))
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 2001, 1000))
    rng = np.random.default_rng(63)
    keys_all, ts_all, vals, got = [], [], [], []
    for step in range(2):
        k = rng.integers(0, nkeys, N).astype(np.uint32)
        ts = np.arange(N, dtype=np.int64) // rate + step * 1000
        v = _signed(rng, N)
        dk = torch.from_numpy(k.view(np.int32)).to(dev)
        dts, dv = torch.from_numpy(ts).to(dev), torch.from_numpy(v).to(dev)
        torch.cuda.synchronize(dev)
        op.processElementsDevice(dk.data_ptr(), dts.data_ptr(), dv.data_ptr(), N)
        got.append(op.processWatermarkArrays(step * 1000 + 999))
        keys_all.append(k)
        ts_all.append(ts)
        vals.append(v)
        del dk, dts, dv
    k = np.concatenate(keys_all).astype(np.int64)
    ts = np.concatenate(ts_all)
    v = np.concatenate(vals)
    comp = (k << 32) | ts  # ts < 2^32 here
    wa = wr = 0.0
    order = np.argsort(comp, kind="stable")
    comp = comp[order]
    vs = v[order]
    del order
    pre = np.concatenate([[0], np.cumsum(vs.astype(np.longdouble))])
    pabs = np.concatenate([[0], np.cumsum(np.abs(vs).astype(np.longdouble))])
    checked = 0
    for a in got:
        kk = a["key"].astype(np.int64) << 32
        lo = np.searchsorted(comp, kk | a["start"], side="left")
        hi = np.searchsorted(comp, kk | a["end"], side="left")
        n, wa_, wr_ = _check(_arrays_rows(a), lo, hi, pre, pabs)
        checked += n
        wa, wr = max(wa, wa_), max(wr, wr_)
    assert checked >= nkeys  # every key emits its [0, 1000) window
    print("keyed: %d windows, worst |err|/sum|x| %.2e, worst |err|/|sum| %.2e" % (checked, wa, wr))
