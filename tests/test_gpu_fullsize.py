"""Oracle parity at the benchmark's own sizes: the streams bench.py times (BASELINE configs C1, C2, C2s, C3) replayed
through the product at full micro-batch size (2^26 / 2^27 tuples per watermark) and through the CPU oracle on the
same inputs, every emitted window compared bit-exactly (start, end, measure, hasValue, every aggregate).

Each stream first runs a sparse warm-up (1 tuple per ms, as bench.py's CPU baselines do) long enough that every
window definition emits during the full-size steps: the 20 s tumbling windows of C2, the 60 s sliding windows of C1
and C3 (SlidingWindow.triggerWindows emits [ws, ws + size) once ws + size <= wm + 1, C/windowType/SlidingWindow.java:
50-57).  C3 covers a pause step (the stream resumes after a 2 s silence: a new session whose start moves down with
the first late tuples, S/SliceManager.java:64-86, SessionWindow.java:40-116), which the product splits into an
event-exact prefix and a one-pass quiet remainder (exact_engine.cpp, push_batch) -- once with the default prefix and
once with scotty_tune("exact_prefix", 4096), so the split itself is oracle-checked.

Inputs are generated on the host (numpy, seeded), copied to HBM and pushed with processElementsDevice, as bench.py
pushes its resident batches; the oracle (oracle/, C++ restatement of SlicingWindowOperator) processes the same
arrays.  Watermark cadence as in bench.py: one per step."""
import numpy as np
import pytest

from helpers import product, build_ops, same_windows
from specs import Tumbling, Sliding, Session, Time, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return product()


def _dev():
    import torch
    return torch.device("cuda", 0)


def _push_both(ops, ora, ts, vals):
    """Push one micro-batch to every product operator (resident in HBM) and to the oracle."""
    import torch
    dts = torch.from_numpy(ts).to(_dev())
    dv = torch.from_numpy(vals).to(_dev())
    torch.cuda.synchronize(_dev())
    for op in ops:
        op.processElementsDevice(dts.data_ptr(), dv.data_ptr(), len(ts))
    failed = ora.processElements(ts, vals)
    return (dts, dv), failed


def _watermark_both(ops, ora, wm, keep):
    exp = ora.processWatermark(wm)
    for op in ops:
        same_windows(op.processWatermark(wm), exp)
    del keep  # the device buffers stay valid until every operator's watermark returned
    return len(exp)


def _run(ops, ora, steps):
    """steps: iterable of (ts, vals, watermark).  Returns the windows compared per step."""
    out = []
    for ts, vals, wm in steps:
        keep, failed = _push_both(ops, ora, ts, vals)
        assert failed == 0
        out.append(_watermark_both(ops, ora, wm, keep))
        for op in ops:
            assert op.droppedCount() == 0
    return out


def test_c2_headline_stream_at_bench_size(pkg):
    """C2 (bench.py headline): 1000 TumblingWindow(Time, randomTumbling(1000,1,20) Random(10)), SUM_I32 + COUNT,
    in-order, maxLateness 1; 21 s sparse warm-up, then 3 steps of 2^27 tuples (1 s of event time each)."""
    B = 1 << 27
    rate = B // 1000
    sizes = pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10)
    gpu, ora = build_ops(dict(windows=[Tumbling(Time, s) for s in sizes], aggs=[SUM, COUNT], lateness=1))
    rng = np.random.default_rng(11)

    def steps():
        ts = np.arange(0, 21000, dtype=np.int64)
        yield ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64).astype(np.int32), 20999
        for s in range(3):
            ts = 21000 + s * 1000 + np.arange(B, dtype=np.int64) // rate
            yield ts, rng.integers(-2**31, 2**31, size=B, dtype=np.int64).astype(np.int32), int(ts[-1])
    n = _run([gpu], ora, steps())
    assert all(k > 0 for k in n[1:]), n
    assert gpu._debug_stat(5) == 1  # the grid path


def test_c2s_north_star_stream_at_bench_size(pkg):
    """C2s (north_star target): 1000 SlidingWindow(size, size/20) of randomTumbling sizes, SUM_I32 + COUNT, 20 % of the
    tuples late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000; 21 s sparse warm-up, 3 steps of 2^27."""
    import importlib
    B = 1 << 27
    rate = B // 1000
    bench = importlib.import_module("bench")
    wins = [Sliding(Time, size, slide) for size, slide in bench.c2s_windows(pkg)]
    gpu, ora = build_ops(dict(windows=wins, aggs=[SUM, COUNT], lateness=1000))
    rng = np.random.default_rng(12)

    def steps():
        ts = np.arange(1, 21000, dtype=np.int64)
        yield ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64).astype(np.int32), 20499
        for s in range(3):
            ts = 21000 + s * 1000 + np.arange(B, dtype=np.int64) // rate
            late = rng.random(B) < 0.2
            d = rng.integers(1, 501, size=B)
            ts = np.where(late, np.maximum(ts - d, 1), ts)
            yield ts, rng.integers(-2**31, 2**31, size=B, dtype=np.int64).astype(np.int32), \
                21000 + s * 1000 + 999 - 500
    n = _run([gpu], ora, steps())
    assert all(k > 1000 for k in n[1:]), n


def test_c1_reference_benchmark_stream_at_bench_size(pkg):
    """C1 (BASELINE configs[0], the reference benchmark's workload): SlidingWindow(Time, 60000, 1000), SUM_I32 of
    java.util.Random(43).nextInt() values, in-order, maxLateness 1; 60 s sparse warm-up, 3 steps of 2^26."""
    B = 1 << 26
    rate = B // 1000
    jr = pkg.workloads.JavaRandomInts(43)
    gpu, ora = build_ops(dict(windows=[Sliding(Time, 60_000, 1_000)], aggs=[SUM], lateness=1))

    def steps():
        ts = np.arange(0, 60_000, dtype=np.int64)
        yield ts, jr.next_ints(len(ts)), 59_999
        for s in range(3):
            ts = 60_000 + s * 1000 + np.arange(B, dtype=np.int64) // rate
            yield ts, jr.next_ints(B), int(ts[-1])
    n = _run([gpu], ora, steps())
    assert all(k >= 1 for k in n), n  # [0,60000) at the warm-up, then the windows of every second


def _c3_ops(pkg, tunes):
    cfg = dict(windows=[Sliding(Time, 60_000, 60), Session(Time, 1000)], aggs=[MIN, MAX], lateness=1000)
    ops = []
    ora = None
    for t in tunes:
        g, o = build_ops(cfg, tune=t)
        ops.append(g)
        ora = ora or o
    return ops, ora


def _c3_steps(B, first_full, last, seed):
    """bench.py's C3 stream: step s covers [t_begin, t_begin + 1000) with t_begin = s*1000 + 1000 + (s//10)*2000 (a
    2 s silence every 10 s: tuples at most 500 ms late leave a 1.5 s gap > the 1 s session gap), 20 % of the tuples late
    by U[1,500] ms (not below t_begin - 500), watermark t_begin + 999 - 500.  Steps before first_full are sparse (1
    tuple per ms, in order), the rest carry B tuples."""
    rng = np.random.default_rng(seed)
    for s in range(last + 1):
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        if s < first_full:
            ts = t_begin + np.arange(1000, dtype=np.int64)
            vals = rng.integers(-2**31, 2**31, size=1000, dtype=np.int64).astype(np.int32)
        else:
            rate = B // 1000
            ts = t_begin + np.arange(B, dtype=np.int64) // rate
            late = rng.random(B) < 0.2
            d = rng.integers(1, 501, size=B)
            ts = np.where(late, np.maximum(ts - d, t_begin - 500), ts)
            vals = rng.integers(-2**31, 2**31, size=B, dtype=np.int64).astype(np.int32)
        yield s, ts, vals, t_begin + 999 - 500


def test_c3_north_star_stream_at_bench_size_with_pause_step(pkg):
    """C3 (BASELINE configs[2]): SlidingWindow(60 s, 60 ms) + SessionWindow(1 s), MIN_I32 + MAX_I32, 20 % late by
    U[1,500] ms, maxLateness 1000.  69 s of sparse warm-up, then steps 69, 70, 71 at 2^26 tuples: 69 and 71 are quiet
    (one pass), 70 resumes after the silence (event-exact prefix, then the quiet remainder).  Two product operators:
    the default first event-exact piece (max(n/32, 2^20) tuples) and scotty_tune("exact_prefix", 4096); both must leave
    exactly the oracle's windows, sliding and session alike, at every watermark."""
    ops, ora = _c3_ops(pkg, [None, {"exact_prefix": 4096}])
    total, verdicts, split = 0, {}, {}
    for s, ts, vals, wm in _c3_steps(1 << 26, 69, 71, seed=13):
        keep, failed = _push_both(ops, ora, ts, vals)
        assert failed == 0
        verdicts[s] = [op._debug_stat(8) for op in ops]
        split[s] = [op._debug_stat(12) for op in ops]
        if s >= 69:
            print("C3 step %d: quiet attempts (XQ_* | why << 8 | first tuple << 24) per operator: %s" % (
                s, [[hex(op._debug_stat(16 + k)) for k in range(op._debug_stat(15))] for op in ops]), flush=True)
        n = _watermark_both(ops, ora, wm, keep)
        if s >= 69:
            assert n > 0, s  # every full step emits sliding windows (and sessions close at the pause)
            total += n
    assert verdicts[71] == [1, 1], verdicts                             # after the pause: quiet, one pass
    assert verdicts[70][0] != 1 and verdicts[70][1] != 1, verdicts      # the pause step is refused ...
    assert split[70][0] >= 1 and split[70][1] >= 1, split               # ... and its remainder committed in one pass
    assert total > 40, total


@pytest.mark.parametrize("prefix", [0, 4096, 65536])
def test_c3_event_prefix_split_reduced(pkg, prefix):
    """The refused-batch split at reduced size (2^20 tuples per step, three pause steps): the event-exact prefix of
    `prefix` tuples (0: the default) then the quiet path on the rest, growing the prefix 4x per further refusal --
    invisible in the results, which must equal the oracle's at every watermark."""
    tune = {"exact_prefix": prefix} if prefix else None
    ops, ora = _c3_ops(pkg, [tune])
    op = ops[0]
    total = 0
    for s, ts, vals, wm in _c3_steps(1 << 20, 25, 61, seed=31 + prefix):
        keep, failed = _push_both(ops, ora, ts, vals)
        assert failed == 0
        if s % 10 == 0:
            print("step %d quiet attempts: %s" % (s, [hex(op._debug_stat(16 + k)) for k in range(op._debug_stat(15))]),
                  flush=True)
        total += _watermark_both(ops, ora, wm, keep)
    assert op._debug_stat(9) > 20      # quiet commits
    print("quiet commits %d, remainder commits %d" % (op._debug_stat(9), op._debug_stat(12)))
    if prefix:  # (the default prefix, max(n/32, 2^20), is the whole 2^20-tuple batch: no split at this size)
        assert op._debug_stat(12) >= 3  # remainders committed after an event-exact prefix (the pause steps)
    assert total > 100
