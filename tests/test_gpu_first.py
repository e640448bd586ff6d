"""SCOTTY_AGG_FIRST on the GPU (grid path) against the oracle: the arrival index of each window's first partial's
tuple -- the tuple whose fields SumAggregation / SumWindowFunction-style combines keep (B/flinkBenchmark/aggregations/
SumAggregation.java:16-18, S/state/AggregateValueState.java:23-31, 55-69) -- bit-exact on random in-order and
out-of-order streams (several pushes per interval, drops, lateness edge skips), on the reference benchmark's own C1
workload, and the retained-firsts list (scotty_first_indices) a shim prunes its payload store with.  Configurations the
column does not run on (sessions, count windows, keyed) fail loudly."""
import numpy as np
import pytest

from helpers import product, build_ops, run_schedule, interval_schedule
from specs import Tumbling, Sliding, FixedBand, Session, Time, Count, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu
FIRST = 10


def _nz(x):
    return x + 1 if x & (x - 1) == 0 else x


@pytest.mark.parametrize("seed", range(10))
def test_first_random_streams_match_oracle(seed):
    rng = np.random.default_rng(9100 + seed)
    wins = []
    for _ in range(int(rng.integers(1, 4))):
        r = rng.random()
        if r < 0.4:
            wins.append(Tumbling(Time, _nz(int(rng.integers(5, 300)))))
        elif r < 0.85:
            size = int(rng.integers(10, 600))
            wins.append(Sliding(Time, size, _nz(int(rng.integers(3, size + 1)))))
        else:
            wins.append(FixedBand(Time, int(rng.integers(0, 2000)), int(rng.integers(1, 1500))))
    aggs = [[SUM, FIRST], [FIRST], [COUNT, FIRST, MIN], [FIRST, SUM, MAX, COUNT]][seed % 4]
    cfg = dict(windows=wins, aggs=aggs, lateness=[1, 5, 100, 1000, None][seed % 5])
    n = int(rng.integers(20_000, 250_000))
    ts, vals = product().workloads.stream(n, [0.5, 2, 10, 40][seed % 4], t0=int(rng.integers(0, 500)),
                                          ooo_frac=[0.0, 0.2, 0.5][seed % 3], max_delay=int(rng.integers(1, 400)),
                                          seed=seed, value_type="i32")
    gpu, ora = build_ops(cfg)
    sched = interval_schedule(ts, int(rng.integers(2, 12)), lag=int(rng.integers(0, 300)),
                              pushes_per_interval=int(rng.integers(1, 4)))
    assert run_schedule(gpu, ora, ts, vals, sched) > 0
    assert gpu._debug_stat(5) == 1  # the grid path


def test_first_on_the_reference_benchmark_workload():
    """C1 (BASELINE configs[0]): SlidingWindow(Time, 60000, 1000), SUM_I32 of Random(43).nextInt(), in order, maxLateness
    1 -- the BenchmarkJob's window and function (SumAggregation keeps the first partial's f0 / f2 / f3) -- at 2000 tuples
    per ms over 70 s, one watermark per second."""
    pkg = product()
    cfg = dict(windows=[Sliding(Time, 60_000, 1000)], aggs=[SUM, FIRST], lateness=1)
    rate, secs = 2000, 70
    ts = np.arange(secs * 1000 * rate, dtype=np.int64) // rate
    vals = pkg.workloads.JavaRandomInts(43).next_ints(len(ts))
    gpu, ora = build_ops(cfg)
    sched = []
    for s in range(secs):
        sched += [("push", s * 1000 * rate, (s + 1) * 1000 * rate), ("wm", s * 1000 + 999)]
    assert run_schedule(gpu, ora, ts, vals, sched) >= secs - 60


def test_first_indices_are_the_retained_slices_firsts():
    """After each watermark, every window a later watermark emits has its FIRST value in the list the previous
    watermark's scotty_first_indices returned, or among the tuples pushed since (what a shim keeps)."""
    pkg = product()
    rng = np.random.default_rng(77)
    cfg = dict(windows=[Sliding(Time, 3000, 250), Tumbling(Time, 700)], aggs=[SUM, FIRST], lateness=800)
    ts, vals = pkg.workloads.stream(400_000, 20, t0=100, ooo_frac=0.3, max_delay=700, seed=5)
    gpu, _ = build_ops(cfg)
    keep, base = set(), 0
    sched = interval_schedule(ts, 20, lag=400, pushes_per_interval=2)
    pushed = 0
    checked = 0
    for step in sched:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                gpu.processElements(ts[lo:hi], vals[lo:hi])
                pushed = hi
        else:
            for w in gpu.processWatermark(step[1]):
                if w.hasValue():
                    f = w.getAggValues()[1]
                    assert f in keep or base <= f < pushed, (f, base, pushed)
                    checked += 1
            got = gpu.firstIndices()
            assert np.all(np.diff(got) > 0) and (len(got) == 0 or got[-1] < pushed)
            keep, base = set(int(x) for x in got), pushed
            assert len(keep) <= gpu.sliceCount()
    assert checked > 50


@pytest.mark.parametrize("windows,keyed", [([Session(Time, 100)], False), ([Tumbling(Count, 100)], False),
                                           ([Tumbling(Time, 100)], True)])
def test_first_refused_off_the_grid_path(windows, keyed):
    pkg = product()
    op = pkg.KeyedSlicingWindowOperator(device=0) if keyed else pkg.SlicingWindowOperator(device=0)
    op.addWindowFunction(SUM)
    op.addWindowFunction(FIRST)
    for w in windows:
        op.addWindowAssigner(w)
    ts = np.arange(1000, dtype=np.int64)
    vals = np.ones(1000, np.int32)
    with pytest.raises(pkg.ScottyError):
        if keyed:
            op.processElements(np.zeros(1000, np.uint32), ts, vals)
        else:
            op.processElements(ts, vals)
        op.processWatermark(2000)
