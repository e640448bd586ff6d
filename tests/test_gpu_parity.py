"""Parity of the MI355X product path (C-ABI -> gfx950 kernels) against the CPU oracle.

Bar: bit-exact for start/end/measure/hasValue and every integer aggregate; SUM_F64 within 1e-6 relative
(BASELINE.json north_star), MIN/MAX_F64 exact.  All cases run on cuda:0 through libscotty_mi355x.so.
"""
import numpy as np
import pytest

import junit_cases
from helpers import product, build_ops, run_schedule, interval_schedule, same_windows
from specs import Tumbling, Sliding, FixedBand, Time, SUM, COUNT, MIN, MAX, SUM_I64, MIN_I64, MAX_I64, \
    SUM_F64, MIN_F64, MAX_F64

pytestmark = pytest.mark.gpu

CF_CASES = junit_cases.TUMBLING_TIME + junit_cases.SLIDING + junit_cases.FIXED_BAND


@pytest.fixture(scope="module")
def pkg():
    return product()


# ---------------------------------------------------------------- the reference's own golden vectors
@pytest.mark.parametrize("case", CF_CASES, ids=lambda c: c.__name__)
def test_junit_golden_values_on_gpu(pkg, case):
    case(lambda: pkg.SlicingWindowOperator(device=0))


# ---------------------------------------------------------------- seeded random configurations
def _not_pow2(x):
    # a power-of-two size/slide makes the reference loop forever (see test_reference_hang_config_rejected)
    return x + 1 if x & (x - 1) == 0 else x


def _random_cfg(rng, value_type):
    wins = []
    for _ in range(int(rng.integers(1, 5))):
        k = int(rng.integers(0, 3))
        if k == 0:
            wins.append(Tumbling(Time, _not_pow2(int(rng.integers(3, 60)))))
        elif k == 1:
            size = int(rng.integers(5, 90))
            wins.append(Sliding(Time, size, _not_pow2(int(rng.integers(2, size + 1)))))
        else:
            wins.append(FixedBand(Time, int(rng.integers(0, 300)), int(rng.integers(1, 200))))
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[value_type]
    aggs = [a for a in aggs if rng.random() < 0.8] or [aggs[0]]
    lateness = [0, 1, 3, 7, 100, 1000, None][int(rng.integers(0, 7))]
    return dict(windows=wins, aggs=aggs, lateness=lateness)


@pytest.mark.parametrize("seed", range(40))
def test_random_streams_match_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    cfg = _random_cfg(rng, vt)
    n = int(rng.integers(1, 60_000))
    rate = [0.2, 1, 3, 20][int(rng.integers(0, 4))]
    ooo = [0.0, 0.05, 0.2, 0.5][int(rng.integers(0, 4))]
    delay = int(rng.integers(1, 400))
    t0 = int(rng.integers(0, 5000))
    ts, vals = product().workloads.stream(n, rate, t0=t0, ooo_frac=ooo, max_delay=delay, seed=seed, value_type=vt)
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, int(rng.integers(1, 8)), lag=int(rng.integers(0, 200)),
                              pushes_per_interval=int(rng.integers(1, 4)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


# ---------------------------------------------------------------- edge semantics of the reference
@pytest.mark.parametrize("win", [Tumbling(Time, 16), Sliding(Time, 100, 64), Tumbling(Time, 1)])
def test_reference_hang_config_rejected(pkg, win):
    """With a power-of-two size/slide, assignNextWindowStart(Long.MAX_VALUE) wraps to exactly Long.MIN_VALUE,
    which calculateNextFixedEdge treats as 'unset' again: the reference spins forever in determineSlices
    (S/StreamSlicer.java:65-69, :103-116).  The oracle reports ORC_ERR_HANG; the product refuses loudly."""
    from oracle.oracle import ERR_HANG, JavaError
    gpu, ora = build_ops(dict(windows=[win, Tumbling(Time, 10)], aggs=[SUM], lateness=5))
    with pytest.raises(JavaError) as ei:
        ora.processElement(1, 100)
    assert ei.value.code == ERR_HANG
    with pytest.raises(pkg.UnsupportedError):
        gpu.processElements(np.array([100], dtype=np.int64), np.array([1], dtype=np.int32))


@pytest.mark.parametrize("ts0,lateness", [(0, 1000), (3, 1000), (999, 1000), (1000, 1000), (5000, 1000),
                                          (7, 1), (10, 1), (12345, 0), (20, 5)])
def test_first_tuple_edge_walk(ts0, lateness):
    """The first in-order tuple walks edges from te-maxLateness (Long.MAX_VALUE wrap, S/StreamSlicer.java:105)."""
    cfg = dict(windows=[Tumbling(Time, 10), Sliding(Time, 30, 7)], aggs=[SUM, COUNT], lateness=lateness)
    ts = np.array([ts0, ts0 + 3, ts0 + 11, ts0 + 2, ts0 + 40, ts0 + 41, ts0 + 90, ts0 + 120], dtype=np.int64)
    vals = np.arange(1, len(ts) + 1, dtype=np.int32)
    gpu, ora = build_ops(cfg)
    run_schedule(gpu, ora, ts, vals, [("push", 0, 4), ("wm", ts0 + 20), ("push", 4, 8), ("wm", ts0 + 200)])


@pytest.mark.parametrize("lateness", [1, 5, 50])
def test_edge_skip_when_stream_jumps(lateness):
    """Edges older than te - maxLateness are skipped on a jump (S/StreamSlicer.java:106)."""
    cfg = dict(windows=[Tumbling(Time, 10), Tumbling(Time, 25)], aggs=[SUM, COUNT, MAX], lateness=lateness)
    ts = np.array([1, 5, 9, 13, 300, 301, 12, 305, 999, 1003, 1010, 2500, 2490, 2600], dtype=np.int64)
    vals = np.arange(len(ts), dtype=np.int32) * 7 - 20
    gpu, ora = build_ops(cfg)
    run_schedule(gpu, ora, ts, vals, [("push", 0, 6), ("push", 6, 11), ("wm", 1000), ("push", 11, 14),
                                      ("wm", 5000)])


def test_windows_added_mid_stream():
    """Window added between micro-batches keeps the pending edge (TumblingWindowOperatorTest dynamic cases)."""
    ts, vals = product().workloads.stream(30_000, 5, t0=17, ooo_frac=0.1, max_delay=40, seed=3)
    gpu, ora = build_ops(dict(windows=[Tumbling(Time, 100)], aggs=[SUM, COUNT], lateness=50))
    run_schedule(gpu, ora, ts, vals, [("push", 0, 10_000), ("wm", int(ts[:10_000].max()) - 30)])
    for op in (gpu, ora):
        op.addWindowAssigner(Sliding(Time, 170, 30))
    run_schedule(gpu, ora, ts, vals, [("push", 10_000, 20_000), ("wm", int(ts[:20_000].max()) - 30)])
    for op in (gpu, ora):
        op.addWindowAssigner(FixedBand(Time, int(ts[20_000]) + 5, 333))
    run_schedule(gpu, ora, ts, vals, [("push", 20_000, 30_000), ("wm", int(ts.max()) + 1000)])


def test_too_late_tuples_are_dropped_and_counted(pkg):
    """Tuples before the oldest retained slice: the reference throws IndexOutOfBoundsException per tuple
    (S/SliceManager.java:75-76); the product drops + counts them and returns SCOTTY_WARN_LATE_DROPPED."""
    cfg = dict(windows=[Tumbling(Time, 10)], aggs=[SUM], lateness=1)
    ts = np.array([100, 150, 200, 120, 5, 210, 3, 260], dtype=np.int64)
    vals = np.ones(len(ts), dtype=np.int32)
    gpu, ora = build_ops(cfg)
    run_schedule(gpu, ora, ts, vals, [("push", 0, 3), ("wm", 190), ("push", 3, 8), ("wm", 400)])
    assert gpu.droppedCount() == 3 and gpu.last_status == pkg.SCOTTY_WARN_LATE_DROPPED


def test_int32_wraparound_sum():
    cfg = dict(windows=[Tumbling(Time, 1000)], aggs=[SUM, COUNT], lateness=1)
    n = 50_000
    ts = np.arange(n, dtype=np.int64) // 10
    vals = np.full(n, 2**31 - 1, dtype=np.int32)
    gpu, ora = build_ops(cfg)
    run_schedule(gpu, ora, ts, vals, [("push", 0, n), ("wm", int(ts.max()) + 2000)])


def test_f64_min_max_nan_and_signed_zero():
    cfg = dict(windows=[Tumbling(Time, 5)], aggs=[MIN_F64, MAX_F64, SUM_F64], lateness=10)
    ts = np.arange(16, dtype=np.int64) * 5 // 4
    vals = np.array([1.0, -0.0, 0.0, 2.0, np.nan, 1.0, 3.0, -5.0, 0.0, -0.0, -0.0, 0.0,
                     np.inf, -np.inf, 1e300, -1e300], dtype=np.float64)
    gpu, ora = build_ops(cfg, "f64")
    assert gpu.processWatermark(0) == [] and ora.processWatermark(0) == []
    gpu.processElements(ts, vals)
    ora.processElements(ts, np.zeros(16, dtype=np.int64), vals)
    a = gpu.processWatermark(100)
    b = ora.processWatermark(100)
    assert len(a) == len(b) == 20
    for x, y in zip(a, b):
        assert x.hasValue() == y.hasValue()
        for p, q in zip(x.getAggValues()[:2], y.getAggValues()[:2]):
            assert (np.isnan(p) and np.isnan(q)) or (p == q and np.signbit(p) == np.signbit(q)), (x, y)


# ---------------------------------------------------------------- benchmark configurations, reduced size
def test_config1_sliding_60s_1s_sum():
    ts, vals = product().workloads.stream(3_000_000, 20, t0=0, seed=43)   # 150 s of event time
    gpu, ora = build_ops(dict(windows=[Sliding(Time, 60_000, 1_000)], aggs=[SUM], lateness=1))
    sched = interval_schedule(ts, 150, lag=0)
    assert run_schedule(gpu, ora, ts, vals, sched) > 0


def test_config2_1000_random_tumbling_sum_count():
    sizes = product().workloads.random_tumbling_sizes(1000, 1, 20, seed=10)
    ts, vals = product().workloads.stream(2_000_000, 50, t0=0, seed=10)   # 40 s
    gpu, ora = build_ops(dict(windows=[Tumbling(Time, s) for s in sizes], aggs=[SUM, COUNT], lateness=1))
    sched = interval_schedule(ts, 40, lag=0)
    assert run_schedule(gpu, ora, ts, vals, sched) > 1000


def test_config3_sliding_1000_concurrent_out_of_order_min_max():
    ts, vals = product().workloads.stream(3_000_000, 25, t0=1000, ooo_frac=0.2, max_delay=500, seed=7)  # 120 s
    gpu, ora = build_ops(dict(windows=[Sliding(Time, 60_000, 60)], aggs=[MIN, MAX, COUNT], lateness=1000))
    sched = interval_schedule(ts, 120, lag=500)
    assert run_schedule(gpu, ora, ts, vals, sched) > 0


def test_large_batch_tumbling_partition_property(pkg):
    """At full micro-batch size (2^25 tuples): tumbling windows partition the in-order stream, so the
    COUNT over all emitted windows equals the tuple count and the wrapped SUMs add up (mod 2^32)."""
    n = 1 << 25
    ts = np.arange(n, dtype=np.int64) // 33_554
    vals = np.random.default_rng(5).integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    op = pkg.SlicingWindowOperator()
    op.addWindowFunction(SUM)
    op.addWindowFunction(COUNT)
    op.addWindowAssigner(Tumbling(Time, 7))
    op.setMaxLateness(1)
    assert op.processWatermark(0) == []   # empty store: lastWatermark := 0, so the next one emits from 0
    op.processElements(ts, vals)
    ws = op.processWatermark(int(ts.max()) + 100)
    cnt = sum(w.getAggValues()[1] for w in ws if w.hasValue())
    tot = sum(w.getAggValues()[0] for w in ws if w.hasValue())
    assert cnt == n
    assert (tot - int(vals.astype(np.int64).sum())) % (1 << 32) == 0


# ---------------------------------------------------------------- watermark path: block summaries / sparse table
@pytest.mark.parametrize("vt", ["i32", "i64", "f64"])
def test_windows_over_many_slice_blocks(vt):
    """Windows spanning thousands of slices (= many 64-slice blocks): prefix-sum differences, sparse-table levels
    and partial head/tail blocks (window_kernels.hip) against the oracle's O(S*W) assembly
    (S/aggregationstore/LazyAggregateStore.java:83-111), out-of-order tuples touching old blocks."""
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    cfg = dict(windows=[Tumbling(Time, 3), Sliding(Time, 5003, 997), Sliding(Time, 20011, 3001),
                        FixedBand(Time, 1234, 40000)], aggs=aggs, lateness=300)
    ts, vals = product().workloads.stream(400_000, 5, t0=11, ooo_frac=0.1, max_delay=250, seed=21, value_type=vt)
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, 12, lag=200, pushes_per_interval=2)
    f64_cols = [0] if vt == "f64" else []
    assert run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols) > 20000


def test_slice_compaction_keeps_window_assembly_exact():
    """More than 2^19 slices over the operator's life: the slice arrays are compacted at a watermark (head moves
    to 0), which re-bases every block summary; windows before and after must stay bit-exact."""
    n = 600_000
    ts = np.arange(n, dtype=np.int64) * 3 + 1
    vals = np.random.default_rng(8).integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    cfg = dict(windows=[Tumbling(Time, 3), Sliding(Time, 9001, 3001)], aggs=[SUM, COUNT, MAX], lateness=10)
    gpu, ora = build_ops(cfg)
    sched = interval_schedule(ts, 14, lag=5)
    assert run_schedule(gpu, ora, ts, vals, sched) > n // 2


def test_watermark_arrays_f64_columns(pkg):
    """processWatermarkArrays returns F64 aggregations as doubles, equal to processWatermark's values."""
    cfg = dict(windows=[Tumbling(Time, 50), Sliding(Time, 200, 70)], aggs=[SUM_F64, MIN_F64, MAX_F64, COUNT],
               lateness=20)
    ts, vals = product().workloads.stream(20_000, 4, t0=3, seed=9, value_type="f64")
    a, _ = build_ops(cfg, "f64")
    b, _ = build_ops(cfg, "f64")
    for op in (a, b):
        op.processElements(ts, vals)
    rows = a.processWatermark(int(ts.max()) + 500)
    arr = b.processWatermarkArrays(int(ts.max()) + 500)
    assert len(rows) == len(arr["start"]) > 0
    for k in range(3):
        assert arr["values"][k].dtype == np.float64
    for i, w in enumerate(rows):
        assert (w.getStart(), w.getEnd(), w.hasValue()) == (arr["start"][i], arr["end"][i], arr["has_value"][i])
        if w.hasValue():
            assert w.getAggValues()[:3] == [arr["values"][k][i] for k in range(3)]
            assert w.getAggValues()[3] == arr["values"][3][i]


def test_device_timing_classes(pkg):
    """scotty_device_timing: every launch group of a grid-path step lands in one class."""
    ts, vals = product().workloads.stream(200_000, 50, t0=0, seed=2)
    op = pkg.SlicingWindowOperator()
    op.addWindowFunction(SUM)
    op.addWindowAssigner(Tumbling(Time, 100))
    op.setMaxLateness(1)
    op.enableTiming(True)
    for lo in range(0, len(ts), 50_000):
        op.processElements(ts[lo:lo + 50_000], vals[lo:lo + 50_000])
        op.processWatermark(int(ts[lo + 49_999]))
    t = op.deviceTiming()
    assert t["ingest"][1] == 4 and t["watermark"][1] == 4
    # the watermark writes its rows straight into host-mapped memory: a result-copy interval exists only where the
    # library fell back to a DMA transfer (no device address for the pinned buffer)
    assert t["result_copy"][1] in (0, 4), t
    assert t["push_other"][1] == 8
    assert all(v[0] > 0 for v in t.values() if v[1] > 0), t


def test_f64_sum_at_bench_scale(pkg):
    """SUM_F64 at the bench's batch size (2 micro-batches of 2^26 tuples, 1000 tumbling windows of 50-1000 ms): the
    grid path's partials reassociate the reference's arrival-order fold (atomicAdd(double) per cell, then slices, then
    windows), so every window is checked against its exactly rounded sum (long double prefix sums on the host) within
    the north_star's 1e-6 relative, and COUNT bit-exactly.  Positive values: no cancellation, so the relative bound
    measures the kernel's rounding alone."""
    import torch
    dev = torch.device("cuda", 0)
    rate = (1 << 26) // 1000
    sizes = [_not_pow2(50 + (x % 951)) for x in pkg.workloads.random_tumbling_sizes()]
    op = pkg.SlicingWindowOperator(device=0, value_type=pkg.VALUE_F64)
    op.addWindowFunction(pkg.AGG_SUM_F64)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for s in sizes:
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    n = 1 << 26
    host_v = []
    rows = []
    for step in range(2):
        ts = torch.arange(n, device=dev, dtype=torch.int64) // rate + step * 1000
        v = torch.rand(n, device=dev, dtype=torch.float64, generator=g) * 1000.0
        torch.cuda.synchronize(dev)
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), n)
        rows += op.processWatermark(step * 1000 + 999)
        host_v.append(v.cpu().numpy())
        del ts, v
    vals = np.concatenate(host_v).astype(np.longdouble)
    pre = np.concatenate([[np.longdouble(0)], np.cumsum(vals)])
    ts_all = np.concatenate([np.arange(n, dtype=np.int64) // rate + k * 1000 for k in range(2)])  # non-decreasing
    checked = 0
    worst = 0.0
    for w in rows:
        lo, hi = np.searchsorted(ts_all, [w.getStart(), w.getEnd()], side="left")
        if hi <= lo:
            assert not w.hasValue()
            continue
        exp_sum, exp_cnt = pre[hi] - pre[lo], hi - lo
        s, c = w.getAggValues()
        assert c == exp_cnt
        rel = abs(float((np.longdouble(s) - exp_sum) / exp_sum))
        worst = max(worst, rel)
        assert rel <= 1e-6, (w.getStart(), w.getEnd(), s, float(exp_sum))
        checked += 1
    assert checked > 1000 and worst < 1e-6


# ---------------------------------------------------------------- every ingest loop of the grid path
@pytest.mark.parametrize("mode", [6, 7, 22, 23])
@pytest.mark.parametrize("seed", range(4))
def test_ingest_loops_match_oracle(mode, seed):
    """The int32 ingest loops scotty_tune("ingest_mode") selects (6 plain, 7 software-pipelined, 22 / 23 the same with
    the DQ2 deferred queue: one DPP scan per step, full-pass folds) on out-of-order streams dense enough that every
    wave queues and folds many out-of-order tuples (the queue's remainder carried across steps, the end-of-range fold
    of a partial pass), against the oracle.  SUM / COUNT and MIN / MAX configurations (mode 23 covers both)."""
    rng = np.random.default_rng(7700 + seed)
    aggs = [[SUM, COUNT], [SUM], [COUNT, MIN, MAX], [MIN, SUM]][seed]
    if mode == 22 and (MIN in aggs or MAX in aggs):
        pytest.skip("mode 22 is the SUM / COUNT loop only")
    cfg = dict(windows=[Sliding(Time, _not_pow2(int(rng.integers(200, 3000))), _not_pow2(int(rng.integers(5, 90)))),
                        Tumbling(Time, _not_pow2(int(rng.integers(30, 700))))], aggs=aggs, lateness=1000)
    n = 1_500_000
    ts, vals = product().workloads.stream(n, 400, t0=100, ooo_frac=[0.2, 0.5, 0.05, 0.3][seed], max_delay=400,
                                          seed=seed, value_type="i32")
    gpu, ora = build_ops(cfg, "i32", tune={"ingest_mode": mode})
    sched = interval_schedule(ts, 4, lag=400, pushes_per_interval=2)
    assert run_schedule(gpu, ora, ts, vals, sched) > 0
