"""Parity of the count-window path (count_common.h / count_kernels.hip: non-keyed operators whose windows are
all context-free COUNT windows, BASELINE configs[4]; chosen with the in-order promise scotty_tune("count_path", 1))
against the oracle, and against the exact engine (the default, which keeps LazySlice record sets)."""
import numpy as np
import pytest

from helpers import product, build_ops, run_schedule, interval_schedule, same_windows
from specs import Tumbling, Sliding, FixedBand, Count, Time, SUM, COUNT, MIN, MAX, SUM_I64, MIN_I64, MAX_I64, \
    SUM_F64, MIN_F64, MAX_F64

pytestmark = pytest.mark.gpu


def _aggs(rng, vt):
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    return [a for a in aggs if rng.random() < 0.6] or [aggs[int(rng.integers(0, 4))]]


def _count_windows(rng, max_size):
    wins = []
    for _ in range(int(rng.integers(1, 5))):
        r = rng.random()
        if r < 0.5:
            wins.append(Tumbling(Count, int(rng.integers(1, max_size))))
        elif r < 0.85:
            size = int(rng.integers(2, max_size))
            wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
        else:
            wins.append(FixedBand(Count, int(rng.integers(0, 3 * max_size)), int(rng.integers(1, 2 * max_size))))
    return wins


def _in_order_stream(rng, n, rate, t0, vt, n_late=0):
    """Non-decreasing timestamps with ties (rate tuples per ms) plus n_late tuples older than every slice
    (the reference throws IndexOutOfBoundsException for them: dropped and counted)."""
    ts = t0 + (np.arange(n, dtype=np.int64) * 1000 // max(1, int(rate * 1000)))
    if vt == "f64":
        vals = rng.normal(0, 1e3, size=n)
    elif vt == "i64":
        vals = rng.integers(-2**40, 2**40, size=n, dtype=np.int64)
    else:
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    if n_late:
        pos = rng.choice(np.arange(n // 4, n), size=n_late, replace=False)
        ts[pos] = t0 - 1 - rng.integers(0, 1000, size=n_late)
    return ts, vals


@pytest.mark.parametrize("seed", range(16))
def test_count_path_matches_oracle(seed):
    rng = np.random.default_rng(12000 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    cfg = dict(windows=_count_windows(rng, [20, 200, 2000][seed % 3]), aggs=_aggs(rng, vt),
               lateness=int(rng.choice([1, 10, 1000])))
    n = int(rng.integers(1000, 60_000))
    ts, vals = _in_order_stream(rng, n, [0.3, 2, 25][seed % 3], int(rng.integers(0, 5000)), vt,
                                n_late=int(rng.integers(0, 5)))
    gpu, ora = build_ops(cfg, vt, tune={"count_path": 1})
    sched = interval_schedule(ts, int(rng.integers(1, 12)), lag=int(rng.integers(0, 50)),
                              pushes_per_interval=int(rng.integers(1, 4)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


@pytest.mark.parametrize("vt", ["i32", "i64", "f64"])
def test_count_path_push_sizes_around_the_step(vt):
    """The count ingest's step pipeline at its boundaries: pushes of 1, 255, 256, 257, 511, 512, 513, 767, 768, 769,
    4095, 4096, 4097 and 70000 tuples (a lone ragged step, one / two / three full steps with and without a ragged
    one, odd and even numbers of full steps per wave), a watermark after every other push, against the oracle."""
    rng = np.random.default_rng(12700 + ["i32", "i64", "f64"].index(vt))
    sizes = [1, 255, 256, 257, 511, 512, 513, 767, 768, 769, 4095, 4096, 4097, 70000]
    n = int(sum(sizes))
    cfg = dict(windows=[Tumbling(Count, 97), Sliding(Count, 700, 300), Tumbling(Count, 5000)],
               aggs=_aggs(np.random.default_rng(1), vt) if vt != "i32" else [SUM, COUNT, MIN, MAX], lateness=10)
    ts, vals = _in_order_stream(rng, n, 2, 1000, vt)
    sched, lo = [], 0
    for i, m in enumerate(sizes):
        sched.append(("push", lo, lo + m))
        lo += m
        if i % 2 == 1:
            sched.append(("wm", int(ts[:lo].max()) - 3))
    sched.append(("wm", int(ts.max())))
    gpu, ora = build_ops(cfg, vt, tune={"count_path": 1})
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


@pytest.mark.parametrize("seed", range(6))
def test_count_path_prefix_sum_kernels_agree(seed):
    """The watermark's prefix sums of SUM / COUNT windows: one workgroup (the default up to 2^16 slices in range) and
    the three-kernel scan (scotty_tune "count_prefix_one" 0) both match the oracle on the same stream."""
    for one in (1, 0):
        rng = np.random.default_rng(12500 + seed)
        cfg = dict(windows=_count_windows(rng, [20, 200, 2000][seed % 3]), aggs=[SUM, COUNT],
                   lateness=int(rng.choice([1, 10, 1000])))
        n = int(rng.integers(20_000, 80_000))
        ts, vals = _in_order_stream(rng, n, [0.3, 2, 25][seed % 3], int(rng.integers(0, 5000)), "i32")
        gpu, ora = build_ops(cfg, "i32", tune={"count_path": 1, "count_prefix_one": one})
        sched = interval_schedule(ts, int(rng.integers(2, 12)), lag=int(rng.integers(0, 50)),
                                  pushes_per_interval=int(rng.integers(1, 4)))
        run_schedule(gpu, ora, ts, vals, sched, value_type="i32")


@pytest.mark.parametrize("seed", range(6))
def test_count_path_out_of_order_never_silently_wrong(pkg, seed):
    """Out-of-order tuples older than their own count slice need LazySlice record moves (S/SliceManager.java:
    77-85): the count path must either match the oracle (the tuples landed in the open slice) or fail loudly."""
    rng = np.random.default_rng(12500 + seed)
    cfg = dict(windows=_count_windows(rng, 300), aggs=[SUM, COUNT, MAX], lateness=1000)
    n = 20_000
    ts, vals = product().workloads.stream(n, 2, t0=1000, ooo_frac=[0.001, 0.05][seed % 2],
                                          max_delay=int(rng.integers(1, 30)), seed=seed)
    gpu, ora = build_ops(cfg, tune={"count_path": 1})
    sched = interval_schedule(ts, 6, lag=40)
    try:
        run_schedule(gpu, ora, ts, vals, sched)
    except pkg.ScottyError as e:
        assert e.code == -2, e  # SCOTTY_ERR_UNSUPPORTED
    # without the in-order promise the operator keeps LazySlice record sets and matches exactly
    gpu, ora = build_ops(cfg)
    run_schedule(gpu, ora, ts, vals, sched)


def test_count_path_equals_exact_engine(pkg):
    """Count path vs the exact engine (tune "count_path" 0) on a 2M-tuple stream: identical rows."""
    rng = np.random.default_rng(12900)
    wins = [Tumbling(Count, 1000), Sliding(Count, 5000, 700), Tumbling(Count, 333), FixedBand(Count, 10_000, 90_000)]
    n = 2_000_000
    ts, vals = _in_order_stream(rng, n, 40, 100, "i32")
    ops = []
    for path in (1, 0):
        op = pkg.SlicingWindowOperator(device=0)
        op.tune("count_path", path)
        for a in (SUM, COUNT, MIN, MAX):
            op.addWindowFunction(a)
        op.setMaxLateness(50)
        for w in wins:
            op.addWindowAssigner(w)
        ops.append(op)
    total = 0
    for step in interval_schedule(ts, 10, lag=5, pushes_per_interval=2):
        if step[0] == "push":
            for op in ops:
                op.processElements(ts[step[1]:step[2]], vals[step[1]:step[2]])
        else:
            a, b = ops[0].processWatermark(step[1]), ops[1].processWatermark(step[1])
            same_windows(a, b)
            total += len(a)
    assert total > 1000


def test_count_config5_reduced():
    """BASELINE configs[4] shape at reduced size: BenchmarkRunner.randomCount(100, 1000, 20000) tumbling count
    windows (java.util.Random(10)), SUM + COUNT, in-order, many pushes and watermarks."""
    pkg = product()
    sizes = pkg.workloads.random_count_sizes(100, 1000, 20000, seed=10)
    cfg = dict(windows=[Tumbling(Count, s) for s in sizes], aggs=[SUM, COUNT], lateness=1)
    n = 400_000
    rng = np.random.default_rng(5)
    ts, vals = _in_order_stream(rng, n, 50, 0, "i32")
    for tune in ({"count_path": 1}, None):
        gpu, ora = build_ops(cfg, tune=tune)
        assert run_schedule(gpu, ora, ts, vals, interval_schedule(ts, 16, lag=0, pushes_per_interval=2)) > 1000


def _time_windows(rng, scale):
    """Steps are never powers of two: assignNextWindowStart(Long.MAX_VALUE) then wraps to Long.MIN_VALUE and the
    reference's first calculateNextFixedEdge loops forever (both sides fail, test_count_path_hang_config)."""
    def step(lo, hi):
        v = int(rng.integers(lo, hi))
        while v & (v - 1) == 0:
            v += 1
        return v
    wins = []
    for _ in range(int(rng.integers(1, 4))):
        r = rng.random()
        if r < 0.4:
            wins.append(Tumbling(Time, step(1, scale)))
        elif r < 0.85:
            size = int(rng.integers(3, 4 * scale))
            wins.append(Sliding(Time, size, min(size, step(1, size + 1))))
        else:
            wins.append(FixedBand(Time, int(rng.integers(0, 20 * scale)), int(rng.integers(1, 10 * scale))))
    return wins


@pytest.mark.parametrize("seed", range(20))
def test_count_and_time_windows_on_count_path_match_oracle(pkg, seed):
    """Count windows plus context-free time windows (SURVEY C5's shape) on the count path: the time edges come
    from the in-order stream (CEngine::time_edges: the first tuple's calculateNextFixedEdge walk, then one
    candidate per union grid point decided by the first tuple reaching it, S/StreamSlicer.java:46-83); triggers
    in registration order with (lastWatermark, watermark) for time windows (S/WindowManager.java:104-118)."""
    rng = np.random.default_rng(13000 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    wins = _count_windows(rng, [20, 200, 2000][seed % 3]) + _time_windows(rng, [30, 300, 3000][(seed // 3) % 3])
    order = rng.permutation(len(wins))
    cfg = dict(windows=[wins[i] for i in order], aggs=_aggs(rng, vt), lateness=int(rng.choice([1, 7, 100, 5000])))
    n = int(rng.integers(1000, 60_000))
    ts, vals = _in_order_stream(rng, n, [0.3, 2, 25, 0.05][seed % 4], int(rng.integers(0, 5000)), vt)
    gpu, ora = build_ops(cfg, vt, tune={"count_path": 1})
    sched = interval_schedule(ts, int(rng.integers(1, 12)), lag=int(rng.integers(0, 50)),
                              pushes_per_interval=int(rng.integers(1, 4)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)
    assert gpu._debug_stat(5) == 3


def test_survey_c5_reduced_matches_oracle(pkg):
    """SURVEY C5 at reduced size: TumblingWindow(Count, 1000) + SlidingWindow(Time, 60000, 1000), SUM + COUNT,
    in-order unique timestamps (tsgap 1..3 ms), a watermark per second of event time."""
    rng = np.random.default_rng(13500)
    cfg = dict(windows=[Tumbling(Count, 1000), Sliding(Time, 60000, 1000)], aggs=[SUM, COUNT], lateness=1)
    n = 300_000
    ts = 5 + np.cumsum(rng.integers(1, 4, size=n)).astype(np.int64)
    vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    gpu, ora = build_ops(cfg, tune={"count_path": 1})
    sched = interval_schedule(ts, int((ts[-1] - ts[0]) // 1000), lag=0, pushes_per_interval=2)
    assert run_schedule(gpu, ora, ts, vals, sched) > 800  # 300 count + 540 time windows
    assert gpu._debug_stat(5) == 3


def test_count_path_aggregate_range_exception_leaves_state(pkg):
    """A count window longer than the time windows keep: clearAfterWatermark removes slices older than watermark -
    maxLateness - the largest clearDelay (S/WindowManager.java:82-95), so a TumblingWindow(Count, 1000) spanning 16 s
    of a one-tuple-per-16-ms stream, watermarks ~2 s apart, loses its start slice to a 10 s sliding window's retention
    and LazyAggregateStore.aggregate throws getSlice(-1) (:83-90; the oracle throws at 23 of the 30 watermarks).  The count path's GC is skipped on the device when the
    aggregation threw (one host synchronisation per watermark): every watermark throws or matches the oracle's, and
    the state after a throw is the reference's."""
    cfg = dict(windows=[Tumbling(Count, 1000), Sliding(Time, 10_000, 1000)], aggs=[SUM, COUNT], lateness=1000)
    n = 4000
    ts = 1000 + np.arange(n, dtype=np.int64) * 16
    vals = np.random.default_rng(3).integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    gpu, ora = build_ops(cfg, tune={"count_path": 1})
    throws = 0
    for step in interval_schedule(ts, 30, lag=0, pushes_per_interval=1):
        if step[0] == "push":
            gpu.processElements(ts[step[1]:step[2]], vals[step[1]:step[2]])
            ora.processElements(ts[step[1]:step[2]], vals[step[1]:step[2]])
            continue
        try:
            got = gpu.processWatermark(step[1])
        except pkg.ScottyError as e:
            assert e.code == -5
            from oracle.oracle import JavaError
            with pytest.raises(JavaError):
                ora.processWatermark(step[1])
            throws += 1
            continue
        same_windows(got, ora.processWatermark(step[1]))
    assert throws == 23
    assert gpu._debug_stat(5) == 3


@pytest.mark.parametrize("lateness", [1, 40, 100_000])
def test_count_path_time_edges_small_pushes(pkg, lateness):
    """One-tuple and few-tuple pushes (the first tuple's edge walk alone, candidates at batch ends), a first
    timestamp far above 0 (edges in (te - maxLateness, te] from the first walk), ties at grid points."""
    rng = np.random.default_rng(13600 + lateness)
    cfg = dict(windows=[Sliding(Count, 7, 3), Tumbling(Time, 10), Sliding(Time, 25, 5)], aggs=[SUM, COUNT, MAX],
               lateness=lateness)
    ts = np.sort(rng.integers(100_000, 100_600, size=3000)).astype(np.int64)
    ts[1000:1010] = ts[1000]  # a run of ties
    vals = rng.integers(-1000, 1000, size=3000).astype(np.int32)
    gpu, ora = build_ops(cfg, tune={"count_path": 1})
    sched, lo = [], 0
    for size in [1, 1, 2, 5, 1, 40, 300, 1, 700, 1950]:
        hi = min(len(ts), lo + size)
        sched += [("push", lo, hi), ("wm", int(ts[hi - 1]) - 3)]  # early ones throw on both sides (getSlice(-1))
        lo = hi
    assert run_schedule(gpu, ora, ts, vals, sched) > 0
    assert gpu._debug_stat(5) == 3


def test_count_path_hang_config(pkg):
    """A time window whose step is a power of two: the reference's first calculateNextFixedEdge yields
    Long.MIN_VALUE forever (S/StreamSlicer.java:53-69); the oracle and the count path both refuse."""
    cfg = dict(windows=[Tumbling(Count, 10), Tumbling(Time, 64)], aggs=[SUM], lateness=1)
    ts = np.arange(100, 200, dtype=np.int64)
    vals = np.ones(len(ts), dtype=np.int32)
    gpu, ora = build_ops(cfg, tune={"count_path": 1})
    with pytest.raises(pkg.ScottyError):
        gpu.processElements(ts, vals)
        gpu.processWatermark(150)
    assert ora.processElements(ts, vals) > 0  # the oracle reports the tuples whose processElement would hang


def test_count_path_time_windows_reject_out_of_order(pkg):
    """Time windows on the count path need the in-order promise: a batch out of timestamp order fails loudly
    (within a batch at the watermark, across batches at the push) instead of slicing on a wrong search."""
    cfg = dict(windows=[Tumbling(Count, 10), Tumbling(Time, 100)], aggs=[SUM], lateness=1000)
    ts = np.arange(1000, 3000, dtype=np.int64)
    vals = np.ones(len(ts), dtype=np.int32)
    bad = ts.copy()
    bad[700], bad[701] = bad[701], bad[700] - 50
    gpu, _ = build_ops(cfg, tune={"count_path": 1})
    gpu.processElements(bad, vals)
    with pytest.raises(pkg.ScottyError) as e:
        gpu.processWatermark(2500)
    assert e.value.code == -2
    gpu, _ = build_ops(cfg, tune={"count_path": 1})
    gpu.processElements(ts[1000:], vals[1000:])
    with pytest.raises(pkg.ScottyError) as e:
        gpu.processElements(ts[:1000], vals[:1000])
        gpu.processWatermark(2500)
    assert e.value.code == -2


@pytest.fixture(scope="module")
def pkg():
    return product()
