"""Parity of the count-window path (count_common.h / count_kernels.hip: non-keyed operators whose windows are
all context-free COUNT windows, BASELINE configs[4]; chosen with the in-order promise scotty_tune("count_path", 1))
against the oracle, and against the exact engine (the default, which keeps LazySlice record sets)."""
import numpy as np
import pytest

from helpers import product, build_ops, run_schedule, interval_schedule, same_windows
from specs import Tumbling, Sliding, FixedBand, Count, SUM, COUNT, MIN, MAX, SUM_I64, MIN_I64, MAX_I64, \
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


@pytest.fixture(scope="module")
def pkg():
    return product()
