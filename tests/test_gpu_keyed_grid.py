"""Parity of the keyed engine's sort-free path (csrc/keyed_grid.hip) on the MI355X.

The path takes in-order keyed batches whose windows are context-free time windows on Eager slices (the Flink
connector's common case, BASELINE configs[3]); keys it cannot take in a batch are deferred whole to the sort +
lane replay, batches it cannot take go there entirely.  Every test compares it with the replay path (tune
"keyed_grid" 0, itself checked against the per-key oracles in test_gpu_exact.py) or with the oracle directly:
window bounds, hasValue and integer aggregates bit-exact, f64 sums within 1e-6 relative (north_star).
Reference: flink-connector/.../KeyedScottyWindowOperator.java:56-86, S/StreamSlicer.java:36-116,
S/SliceManager.java:27-87."""
import os

import numpy as np
import pytest

from helpers import product, interval_schedule, KeyedOracle, same_keyed_windows, same_keyed_arrays
from specs import Tumbling, Sliding, FixedBand, Time, SUM, COUNT, MIN, MAX, SUM_I64, MIN_I64, MAX_I64, \
    SUM_F64, MIN_F64, MAX_F64

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return product()


def _nz(x):  # a power-of-two size/slide makes the reference loop forever; avoid it in random configs
    return x + 1 if x & (x - 1) == 0 else x


def _aggs(rng, vt):
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    return [a for a in aggs if rng.random() < 0.6] or [aggs[0]]


def _make(pkg, vt, wins, aggs, lateness, kg):
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]
    op = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
    op.tune("keyed_grid", 1 if kg else 0)
    op.tune("keyed_grid_chunk", 0)  # chunk many-cell pushes however small (the default leaves small ones to replay)
    if kg and os.environ.get("SCOTTY_TEST_KG_VARIANT"):  # run the suite against a kernel variant (A/B candidates)
        op.tune("keyed_grid_variant", int(os.environ["SCOTTY_TEST_KG_VARIANT"]))
    for a in aggs:
        op.addWindowFunction(a)
    op.setMaxLateness(lateness)
    for w in wins:
        op.addWindowAssigner(w)
    return op


def _random_windows(rng):
    wins = []
    for _ in range(int(rng.integers(1, 4))):
        r = rng.random()
        if r < 0.15:
            wins.append(FixedBand(Time, int(rng.integers(0, 4000)), int(rng.integers(100, 3000))))
        elif r < 0.55:
            wins.append(Tumbling(Time, _nz(int(rng.integers(20, 800)))))
        else:
            size = int(rng.integers(50, 3000))
            wins.append(Sliding(Time, size, _nz(int(rng.integers(20, size + 1)))))
    return wins


def _run_pair(pkg, vt, wins, aggs, lateness, keys, ts, vals, sched, f64_cols):
    """Feed both paths the same schedule; compare every watermark's rows.  Returns (rows, pushes taken by the
    sort-free path, pushes with deferred keys)."""
    kg, rp = _make(pkg, vt, wins, aggs, lateness, True), _make(pkg, vt, wins, aggs, lateness, False)
    tw = _make(pkg, vt, wins, aggs, lateness, False) if f64_cols else None  # |x|-fed: sum |x| per row
    total, used, deferred = 0, 0, 0
    for step in sched:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi <= lo:
                continue
            for op in (kg, rp):
                op.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            if tw is not None:
                tw.processElements(keys[lo:hi], ts[lo:hi], np.abs(vals[lo:hi]))
            path = kg._debug_stat(2)
            used += path >= 1
            deferred += path == 2
            assert rp._debug_stat(2) == 0
        else:
            exp = rp.processWatermarkArrays(step[1])
            sc = tw.processWatermarkArrays(step[1]) if tw is not None else None
            total += same_keyed_arrays(kg.processWatermarkArrays(step[1]), exp, f64_cols=f64_cols, scale=sc)
            assert kg.droppedCount() == rp.droppedCount()
    assert kg.keyCount() == rp.keyCount()
    return total, used, deferred


@pytest.mark.parametrize("seed", range(16))
def test_sort_free_path_equals_replay(pkg, seed):
    """Random context-free windows, lateness 0..100000, in-order keyed streams with idle periods, a key set that
    grows over the stream (new keys are deferred to the replay path), pushes that cover one to many grid cells."""
    rng = np.random.default_rng(8800 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    wins = _random_windows(rng)
    aggs = _aggs(rng, vt)
    lateness = int(rng.choice([0, 1, 7, 300, 100_000]))
    n = int(rng.integers(20_000, 400_000))
    rate = [0.5, 3, 20, 100][seed % 4]
    gaps = [(int(i), int(rng.integers(10, 5000))) for i in range(int(rng.integers(2000, 50_000)), n, 60_000)]
    ts, vals = product().workloads.stream(n, rate, t0=int(rng.integers(0, 3000)), seed=seed, value_type=vt,
                                          gaps=gaps)
    nkeys = int(rng.choice([1, 7, 300, 5000, 40_000]))
    grow = np.minimum(nkeys, 1 + np.arange(n) // int(rng.integers(1, 40)))  # new keys keep arriving
    keys = (rng.integers(0, 1 << 30, size=n) % grow).astype(np.uint32) * 7919
    sched = interval_schedule(ts, int(rng.integers(3, 20)), lag=int(rng.integers(0, 200)),
                              pushes_per_interval=int(rng.integers(1, 4)))
    f64_cols = [i for i, a in enumerate(aggs) if a == SUM_F64]
    total, used, _ = _run_pair(pkg, vt, wins, aggs, lateness, keys, ts, vals, sched, f64_cols)
    assert used > 0 or lateness == 0  # maxLateness 0 makes the slices Lazy (SliceFactory): not this path


@pytest.mark.parametrize("seed", range(6))
def test_sort_free_path_matches_per_key_oracles(pkg, seed):
    rng = np.random.default_rng(8900 + seed)
    vt = ["i32", "i64", "f64"][seed % 3]
    wins = _random_windows(rng)
    aggs = _aggs(rng, vt)
    lateness = int(rng.choice([1, 3, 50, 2000]))
    n = int(rng.integers(3000, 20_000))
    ts, vals = product().workloads.stream(n, [1, 2, 4][seed % 3], t0=int(rng.integers(0, 500)), seed=seed,
                                          value_type=vt)
    keys = rng.integers(0, int(rng.choice([3, 40, 300])), size=n).astype(np.uint32)
    cfg = dict(windows=wins, aggs=aggs, lateness=lateness)
    ora = KeyedOracle(cfg)
    op = _make(pkg, vt, wins, aggs, lateness, True)
    f64_cols = [i for i, a in enumerate(aggs) if a == SUM_F64]
    used = total = 0
    for step in interval_schedule(ts, int(rng.integers(4, 12)), lag=int(rng.integers(0, 100)), pushes_per_interval=2):
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                op.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                ora.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                used += op._debug_stat(2) >= 1
        else:
            total += same_keyed_windows(op.processWatermark(step[1]), ora.processWatermark(step[1]), f64_cols=f64_cols)
    assert used > 0


def test_sort_free_defers_new_and_long_walk_keys(pkg):
    """A push with new keys: the known keys stay on the sort-free path, the new keys' tuples are gathered in arrival
    order and replayed.  A key idle for a long time under a large lateness would append more than KG_EMAX empty
    slices in one batch: deferred too."""
    wins, aggs = [Tumbling(Time, 10)], [SUM, COUNT]
    kg, rp = _make(pkg, "i32", wins, aggs, 100_000, True), _make(pkg, "i32", wins, aggs, 100_000, False)

    def push(keys, ts, vals):
        for op in (kg, rp):
            op.processElements(np.asarray(keys, np.uint32), np.asarray(ts, np.int64), np.asarray(vals, np.int32))

    def check(wm):
        exp = {}
        for k, w in rp.processWatermark(wm):
            exp.setdefault(k, []).append(w)
        return same_keyed_windows(kg.processWatermark(wm), exp)

    rng = np.random.default_rng(3)
    push(np.arange(100), np.full(100, 5), rng.integers(-9, 9, 100))           # 100 new keys: replay path
    assert kg._debug_stat(2) == 0
    ks = np.concatenate([np.arange(100), np.arange(100, 150)])
    push(ks, np.full(150, 17), rng.integers(-9, 9, 150))                       # 50 new keys among 150
    assert kg._debug_stat(2) == 2 and kg._debug_stat(3) == 50 and kg._debug_stat(4) == 100
    push(np.arange(150), np.full(150, 25), rng.integers(-9, 9, 150))           # all known: sort-free only
    assert kg._debug_stat(2) == 1 and kg._debug_stat(4) == 150
    check(30)
    push([0, 1, 2, 3], [2000, 2000, 2001, 2003], [1, 2, 3, 4])                 # 0..3 idle for ~2 s: > 8 edges
    assert kg._debug_stat(2) == 2 and kg._debug_stat(3) == 4
    push(np.arange(4, 150), np.full(146, 2010), np.ones(146))
    check(2100)


def test_sort_free_unsorted_batch_goes_to_replay(pkg):
    """A batch one grid cell wide with one tuple out of order: the scatter sees it, nothing commits, the whole batch
    is replayed (a batch over many cells is cut into chunks, each checked on its own)."""
    wins, aggs = [Sliding(Time, 2000, 1000)], [SUM, MAX]
    kg, rp = _make(pkg, "i32", wins, aggs, 50, True), _make(pkg, "i32", wins, aggs, 50, False)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 50, 4000).astype(np.uint32)
    ts = np.arange(4000, dtype=np.int64) // 4
    vals = rng.integers(-100, 100, 4000).astype(np.int32)
    for op in (kg, rp):
        op.processElements(keys[:2000], ts[:2000], vals[:2000])
    t2 = ts[2000:].copy()
    t2[[10, 11]] = t2[[11, 10]] + np.array([0, 3])  # one tuple 3 ms late: the batch is not in order
    for op in (kg, rp):
        op.processElements(keys[2000:], t2, vals[2000:])
    assert kg._debug_stat(2) == 0
    exp = {}
    for k, w in rp.processWatermark(1999):  # [0, 2000) of every key
        exp.setdefault(k, []).append(w)
    assert same_keyed_windows(kg.processWatermark(1999), exp) > 0


def test_sort_free_config4_full_size(pkg):
    """C4 at the bench's size: 2^26 tuples over 2^20 uniform keys per second of event time, SlidingWindow(60 s, 1 s)
    SUM_I32 + COUNT, maxLateness 1.  Second 0 creates the keys (replay path), seconds 1 and 2 run sort-free.  At
    wm = 59999 every key emits exactly [0, 60000) (SlidingWindow.triggerWindows, C/windowType/SlidingWindow.java:
    50-57), holding all three seconds: COUNT = the key's tuples, SUM = their int32-wrapped sum."""
    n, nk = 1 << 26, 1 << 20
    rng = np.random.default_rng(44)
    op = pkg.KeyedSlicingWindowOperator()
    op.addWindowFunction(SUM)
    op.addWindowFunction(COUNT)
    op.setMaxLateness(1)
    op.addWindowAssigner(Sliding(Time, 60_000, 1_000))
    cnt = np.zeros(nk, np.int64)
    tot = np.zeros(nk, np.float64)
    paths = []
    for s in range(3):
        keys = rng.integers(0, nk, size=n, dtype=np.uint32)
        ts = s * 1000 + np.arange(n, dtype=np.int64) // (n // 1000)
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
        op.processElements(keys, ts, vals)
        paths.append(op._debug_stat(2))
        cnt += np.bincount(keys, minlength=nk)
        tot += np.bincount(keys, weights=vals.astype(np.float64), minlength=nk)
    assert paths[1:] == [1, 1], paths
    r = op.processWatermarkArrays(59_999)
    k = r["key"].astype(np.int64)
    assert len(k) == op.keyCount() == int((cnt > 0).sum())
    assert (r["start"] == 0).all() and (r["end"] == 60_000).all()
    assert np.array_equal(r["values"][1], cnt[k])
    wrapped = ((tot.astype(np.int64) + 2**31) % 2**32) - 2**31  # |sum| < 2^53: the float64 bincount is exact
    assert np.array_equal(r["values"][0], wrapped[k])
