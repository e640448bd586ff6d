"""Parity of the exact engine (session windows, count windows, keyed operators) on the MI355X against the
CPU oracle: bit-exact window bounds, hasValue and integer aggregates (f64 sums within 1e-6 relative).

Reference behaviour exercised: SessionWindow.SessionContext (C/windowType/SessionWindow.java:40-116),
SliceManager.checkSliceEdges / splitSlice on out-of-order tuples (S/SliceManager.java:89-192), count
edges (S/StreamSlicer.java:37-44, :88-101), count triggers (S/WindowManager.java:109-115) and the keyed
connector's per-key operators (flink-connector/.../KeyedScottyWindowOperator.java:56-86)."""
import numpy as np
import pytest

import junit_cases
from helpers import product, build_ops, run_schedule, interval_schedule, KeyedOracle, same_keyed_windows, same_keyed_arrays
from specs import Tumbling, Sliding, Session, FixedBand, Time, Count, SUM, COUNT, MIN, MAX, SUM_I64, \
    MIN_I64, MAX_I64, SUM_F64, MIN_F64, MAX_F64, INVERTIBLE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return product()


# ---------------------------------------------------------------- the reference's golden values
@pytest.mark.parametrize("case", junit_cases.SESSION + [junit_cases.tumbling_inOrderTestCount],
                         ids=lambda c: c.__name__)
def test_junit_session_and_count_golden_values_on_gpu(pkg, case):
    case(lambda: pkg.SlicingWindowOperator(device=0))


@pytest.mark.parametrize("case", [junit_cases.tumbling_outOfOrderOrderTestCount,
                                  junit_cases.tumbling_outOfOrderOrderTestCount3], ids=lambda c: c.__name__)
def test_junit_lazy_count_out_of_order_on_gpu(pkg, case):
    """Out-of-order tuples with count windows move LazySlice records (the count-shift loop, S/SliceManager.java:
    77-85; LazySlice.dropLastElement / prependElement, S/slice/LazySlice.java:29-44) -- on the GPU."""
    case(lambda: pkg.SlicingWindowOperator(device=0))


def test_junit_lambda_without_gpu_kind_fails_loudly(pkg):
    """The test-only (a,b)->a-b function (TumblingWindowOperatorTest.java:212) has no GPU kind: loud, no CPU
    fallback."""
    with pytest.raises(pkg.ScottyError):
        junit_cases.tumbling_outOfOrderOrderTestCount2(lambda: pkg.SlicingWindowOperator(device=0))


# ---------------------------------------------------------------- LazySlice record sets (out-of-order, Lazy slices)
def _lazy_aggs(rng, vt, invertible):
    if invertible:  # InvertibleAggregateFunction sums / counts (removal by liftAndInvert)
        base = {"i32": [SUM, COUNT], "i64": [SUM_I64, COUNT], "f64": [SUM_F64, COUNT]}[vt]
        return [a | INVERTIBLE for a in base if rng.random() < 0.8] or [base[0] | INVERTIBLE]
    return _aggs(rng, vt)


@pytest.mark.parametrize("seed", range(24))
def test_out_of_order_count_windows_match_oracle(seed):
    """Random count-window operators (plus time / session windows) on out-of-order streams with duplicate
    timestamps: every out-of-order tuple shifts the last record of each later LazySlice, the TreeSet drops records
    of equal ts, non-invertible functions recompute from the record set (S/state/AggregateValueState.java:33-49)."""
    rng = np.random.default_rng(9700 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    wins = [Tumbling(Count, int(rng.integers(1, 40)))]
    if rng.random() < 0.5:
        size = int(rng.integers(2, 60))
        wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
    if rng.random() < 0.4:
        wins.append(Tumbling(Time, _nz(int(rng.integers(5, 100)))))
    if rng.random() < 0.25:
        wins.append(Session(Time, int(rng.integers(5, 100))))
    rng.shuffle(wins)
    aggs = _lazy_aggs(rng, vt, invertible=seed % 3 == 2)
    cfg = dict(windows=wins, aggs=aggs, lateness=int(rng.choice([10, 100, 1000])))
    n = int(rng.integers(200, 6000))
    ts, vals = product().workloads.stream(n, [0.5, 1, 3, 8][seed % 4], t0=int(rng.integers(0, 500)),
                                          ooo_frac=[0.02, 0.1, 0.3][seed % 3], max_delay=int(rng.integers(1, 60)),
                                          seed=seed, value_type=vt, gaps=_gaps(rng, n, 400, 10, 150))
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, int(rng.integers(1, 6)), lag=int(rng.integers(0, 60)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a & 0xFFFF == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


@pytest.mark.parametrize("seed", range(12))
def test_lazy_session_slices_match_oracle(seed):
    """maxLateness <= 0 makes every slice a LazySlice (S/slice/SliceFactory.java:17-22): out-of-order session
    tuples split / shift / merge slices and move records across the edges (S/SliceManager.java:89-192)."""
    rng = np.random.default_rng(9900 + seed)
    vt = ["i32", "i64", "i32", "f64"][seed % 4]
    cfg = _session_cfg(rng, vt)
    cfg["lateness"] = int(rng.choice([0, -5]))
    cfg["aggs"] = _lazy_aggs(rng, vt, invertible=seed % 4 == 3)
    n = int(rng.integers(100, 5000))
    gaps = _gaps(rng, n, int(rng.integers(50, 800)), 50, 600)
    ts, vals = product().workloads.stream(n, [0.2, 1, 4][seed % 3], t0=int(rng.integers(0, 3000)),
                                          ooo_frac=[0.05, 0.2][seed % 2], max_delay=int(rng.integers(1, 200)),
                                          seed=seed, value_type=vt, gaps=gaps)
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, int(rng.integers(1, 6)), lag=int(rng.integers(0, 200)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a & 0xFFFF == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


def _nz(x):  # a power-of-two size/slide makes the reference loop forever; avoid it in random configs
    return x + 1 if x & (x - 1) == 0 else x


def _aggs(rng, vt):
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    return [a for a in aggs if rng.random() < 0.7] or [aggs[0]]


def _session_cfg(rng, vt):
    wins = [Session(Time, int(rng.integers(3, 300)))]
    if rng.random() < 0.3:
        wins.append(Session(Time, int(rng.integers(3, 300))))
    for _ in range(int(rng.integers(0, 3))):
        if rng.random() < 0.5:
            wins.append(Tumbling(Time, _nz(int(rng.integers(5, 200)))))
        else:
            size = int(rng.integers(10, 300))
            wins.append(Sliding(Time, size, _nz(int(rng.integers(3, size + 1)))))
    rng.shuffle(wins)
    return dict(windows=wins, aggs=_aggs(rng, vt), lateness=int(rng.choice([1, 5, 50, 500, 1000])))


def _gaps(rng, n, every, lo, hi):
    return [(int(i), int(rng.integers(lo, hi))) for i in range(every, n, every)]


@pytest.mark.parametrize("seed", range(24))
def test_session_streams_match_oracle(seed):
    rng = np.random.default_rng(7000 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    cfg = _session_cfg(rng, vt)
    n = int(rng.integers(100, 20_000))
    rate = [0.05, 0.3, 1, 5][int(rng.integers(0, 4))]
    gaps = _gaps(rng, n, int(rng.integers(50, 2000)), 50, 800)
    ooo = [0.0, 0.05, 0.2][int(rng.integers(0, 3))]
    ts, vals = product().workloads.stream(n, rate, t0=int(rng.integers(0, 3000)), ooo_frac=ooo,
                                          max_delay=int(rng.integers(1, 300)), seed=seed, value_type=vt, gaps=gaps)
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, int(rng.integers(1, 10)), lag=int(rng.integers(0, 300)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols)


@pytest.mark.parametrize("seed", range(12))
def test_count_windows_in_order_match_oracle(seed):
    rng = np.random.default_rng(9100 + seed)
    wins = [Tumbling(Count, int(rng.integers(1, 50)))]
    if rng.random() < 0.5:
        size = int(rng.integers(2, 60))
        wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
    if rng.random() < 0.5:
        wins.append(Tumbling(Time, _nz(int(rng.integers(5, 100)))))
    if rng.random() < 0.3:
        wins.append(Session(Time, int(rng.integers(5, 100))))
    cfg = dict(windows=wins, aggs=[SUM, COUNT, MAX], lateness=int(rng.choice([1, 10, 1000])))
    n = int(rng.integers(10, 5000))
    ts, vals = product().workloads.stream(n, [0.5, 1, 3][seed % 3], t0=int(rng.integers(0, 500)), seed=seed,
                                          gaps=_gaps(rng, n, 300, 10, 200))
    gpu, ora = build_ops(cfg)
    sched = interval_schedule(ts, int(rng.integers(1, 6)), lag=int(rng.integers(0, 20)))
    run_schedule(gpu, ora, ts, vals, sched)


@pytest.mark.parametrize("seed", range(8))
def test_batch_parallel_path_equals_serial_replay(pkg, seed):
    """The batch-parallel non-keyed path (exact_batch.hip) and the single-wavefront replay (exact_kernels.hip)
    must leave identical results -- larger streams than the oracle comparisons, many events and segments."""
    rng = np.random.default_rng(4400 + seed)
    cfg = _session_cfg(rng, "i32")
    n = 400_000
    gaps = _gaps(rng, n, int(rng.integers(5_000, 50_000)), 100, 3000)
    ts, vals = product().workloads.stream(n, [2, 10, 40][seed % 3], t0=500, ooo_frac=[0.05, 0.2][seed % 2],
                                          max_delay=int(rng.integers(10, 600)), seed=seed, gaps=gaps)
    ops = []
    for serial in (0, 1):
        op = pkg.SlicingWindowOperator(device=0)
        op.tune("exact_serial", serial)
        for a in cfg["aggs"]:
            op.addWindowFunction(a)
        op.setMaxLateness(cfg["lateness"])
        for w in cfg["windows"]:
            op.addWindowAssigner(w)
        ops.append(op)
    sched = interval_schedule(ts, 6, lag=300, pushes_per_interval=2)
    from helpers import same_windows
    for step in sched:
        if step[0] == "push":
            for op in ops:
                op.processElements(ts[step[1]:step[2]], vals[step[1]:step[2]])
        else:
            a, b = ops[0].processWatermark(step[1]), ops[1].processWatermark(step[1])
            same_windows(a, b)
            assert ops[0].droppedCount() == ops[1].droppedCount()


@pytest.mark.parametrize("seed", range(12))
def test_quiet_path_equals_event_exact_path_and_replay(pkg, seed):
    """The one-pass quiet path (exact_quiet.hip: grid ingest into cells + device verdict) must leave exactly the
    windows of the event-exact batch path (exact_batch.hip) and of the single-wavefront replay, on session streams
    whose pauses and out-of-order tuples make some batches quiet and others not; both verdicts must occur."""
    rng = np.random.default_rng(8800 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    cfg = _session_cfg(rng, vt)
    n = 300_000
    gaps = _gaps(rng, n, int(rng.integers(20_000, 80_000)), 100, 3000)
    ts, vals = product().workloads.stream(n, [2, 10, 40][seed % 3], t0=500, ooo_frac=[0.05, 0.2][seed % 2],
                                          max_delay=int(rng.integers(10, 600)), seed=seed, value_type=vt, gaps=gaps)
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]
    ops = []
    for knob, val in (("exact_quiet", 1), ("exact_quiet", 0), ("exact_serial", 1)):
        op = pkg.SlicingWindowOperator(device=0, value_type=vtc)
        op.tune(knob, val)
        for a in cfg["aggs"]:
            op.addWindowFunction(a)
        op.setMaxLateness(cfg["lateness"])
        for w in cfg["windows"]:
            op.addWindowAssigner(w)
        ops.append(op)
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    sched = interval_schedule(ts, 12, lag=300, pushes_per_interval=3)
    from helpers import same_windows, abs_twin
    twin = abs_twin(cfg) if f64_cols else None  # sum |x| per window (helpers.F64_REL)
    quiet, event, why = 0, 0, []
    for step in sched:
        if step[0] == "push":
            for op in ops:
                op.processElements(ts[step[1]:step[2]], vals[step[1]:step[2]])
            if twin is not None and step[2] > step[1]:
                twin.processElements(ts[step[1]:step[2]], np.zeros(step[2] - step[1], np.int64),
                                     np.abs(vals[step[1]:step[2]]))
            v = ops[0]._debug_stat(8)
            quiet += v == 1
            event += v > 1
            why.append((v, ops[0]._debug_stat(11)))
        else:
            a, b, c = (op.processWatermark(step[1]) for op in ops)
            sc = None
            if twin is not None:
                sc = [w.getAggValues() if w.hasValue() else [0.0] * len(cfg["aggs"])
                      for w in twin.processWatermark(step[1])]
            same_windows(a, b, f64_cols=f64_cols, scale=sc)
            same_windows(a, c, f64_cols=f64_cols, scale=sc)
            assert ops[0].droppedCount() == ops[2].droppedCount()
    assert quiet > 0, ("no batch took the quiet path", cfg, why)
    assert event > 0, ("no batch needed the event-exact path", why)


def test_config3_full_size_quiet_path_equals_replay(pkg):
    """BASELINE configs[2] (C3) at the benchmark's batch size class: SlidingWindow(60 s, 60 ms) + SessionWindow(1 s),
    MIN/MAX, 20 % out-of-order by U[1,500] ms, 2^24 tuples per full step, a 2 s pause every 10 s of event time (the
    session closes: the silence left by tuples up to 500 ms late exceeds the gap), generated on the device like
    bench.py's C3 leg.  68 s of sparse warm-up (1 tuple per ms) first, so the full steps 68-70 emit the 60 s sliding
    windows (ws + size <= wm + 1, C/windowType/SlidingWindow.java:50-57) besides the sessions; step 70 resumes after a
    pause.  Quiet path (default) == event-exact batch path == single-wavefront replay (~23 s per full step), window by
    window, every step, and all three == the oracle."""
    import torch
    from oracle.oracle import OracleOperator
    dev = torch.device("cuda", 0)
    batch = 1 << 24
    rate = batch // 1000
    g = torch.Generator(device=dev)
    g.manual_seed(17)
    ops = []
    for knob, val in (("exact_quiet", 1), ("exact_quiet", 0), ("exact_serial", 1)):
        op = pkg.SlicingWindowOperator(device=0)
        op.tune(knob, val)
        ops.append(op)
    ora = OracleOperator()
    for op in ops + [ora]:
        op.addWindowFunction(MIN)
        op.addWindowFunction(MAX)
        op.addWindowFunction(COUNT)
        op.setMaxLateness(1000)
        op.addWindowAssigner(Sliding(Time, 60_000, 60))
        op.addWindowAssigner(Session(Time, 1000))
    from helpers import same_windows
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    quiet, event, rows, sliding = 0, 0, 0, 0
    import time
    for s in range(71):
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        if s < 68:
            ts = torch.arange(1000, device=dev, dtype=torch.int64) + t_begin
            v = torch.randint(-2**31, 2**31, (1000,), device=dev, dtype=torch.int32, generator=g)
        else:
            ts = base + t_begin
            late = torch.rand(batch, device=dev, generator=g) < 0.2
            d = torch.randint(1, 501, (batch,), device=dev, generator=g)
            ts = torch.where(late, torch.clamp(ts - d, min=t_begin - 500), ts).contiguous()
            v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        n = ts.numel()
        tt = []
        for op in ops:
            t0 = time.perf_counter()
            op.processElementsDevice(ts.data_ptr(), v.data_ptr(), n)
            op.sync()
            tt.append(round(time.perf_counter() - t0, 3))
        assert ora.processElements(ts.cpu().numpy(), v.cpu().numpy()) == 0
        if s >= 68:
            verdict = ops[0]._debug_stat(8)
            print("C3 full-size step %d: verdict %d, push s (quiet, event, serial) %s" % (s, verdict, tt), flush=True)
            quiet += verdict == 1
            event += verdict > 1
        wm = t_begin + (n - 1) // (rate if s >= 68 else 1) - 500
        a, b, c = (op.processWatermark(wm) for op in ops)
        exp = ora.processWatermark(wm)
        same_windows(a, b)
        same_windows(a, c)
        same_windows(a, exp)
        if s >= 68:
            rows += len(a)
            sliding += sum(1 for w in a if w.getEnd() - w.getStart() == 60_000)
    assert quiet >= 1 and event >= 1, (quiet, event)
    assert sliding > 30 and rows > sliding, (rows, sliding)


@pytest.mark.parametrize("vt", ["i32", "i64", "f64"])
def test_exact_engine_window_assembly_from_block_summaries(vt):
    """One operator on the exact engine (a session window beside long sliding windows): windows over hundreds of
    slices are assembled from 64-slice block summaries (exact_kernels.hip wm_blocks_kernel / agg_row), the blocks at a
    run's ends slice by slice; out-of-order tuples and session edits change old blocks between watermarks."""
    aggs = {"i32": [MIN, MAX, SUM, COUNT], "i64": [MAX_I64, SUM_I64, MIN_I64], "f64": [SUM_F64, MIN_F64, MAX_F64, COUNT]}
    cfg = dict(windows=[Sliding(Time, 9001, 13), Session(Time, 400), Sliding(Time, 2003, 7)], aggs=aggs[vt],
               lateness=600)
    n = 400_000
    gaps = [(i, 900) for i in range(60_000, n, 90_000)]
    ts, vals = product().workloads.stream(n, 8, t0=100, ooo_frac=0.2, max_delay=300, seed=61, value_type=vt,
                                          gaps=gaps)
    gpu, ora = build_ops(cfg, vt)
    sched = interval_schedule(ts, 30, lag=300, pushes_per_interval=2)
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    assert run_schedule(gpu, ora, ts, vals, sched, value_type=vt, f64_cols=f64_cols) > 2000


def test_session_tumbling_mixed_config3_reduced():
    """BASELINE configs[2] at reduced size: sliding + session, 20 % out-of-order (TimeStampGenerator-like,
    delay U[1,500]), MIN/MAX; session silences every ~10 s of event time."""
    n = 600_000
    rate = 25
    gaps = [(i, 1500) for i in range(250_000 // 1, n, 250_000)]
    ts, vals = product().workloads.stream(n, rate, t0=1000, ooo_frac=0.2, max_delay=500, seed=33, gaps=gaps)
    cfg = dict(windows=[Sliding(Time, 6000, 60), Session(Time, 1000)], aggs=[MIN, MAX, COUNT], lateness=1000)
    gpu, ora = build_ops(cfg)
    sched = interval_schedule(ts, 24, lag=500)
    assert run_schedule(gpu, ora, ts, vals, sched) > 0


# ---------------------------------------------------------------- keyed
def _keyed_run(pkg, cfg, keys, ts, vals, sched, vt="i32", f64_cols=()):
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]
    gpu = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
    for a in cfg["aggs"]:
        gpu.addWindowFunction(a)
    if cfg.get("lateness") is not None:
        gpu.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        gpu.addWindowAssigner(w)
    ora = KeyedOracle(cfg)
    twin = KeyedOracle(cfg) if vt == "f64" and f64_cols else None  # sum |x| per window (helpers.F64_REL)
    total = 0
    for step in sched:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                gpu.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                ora.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                if twin is not None:
                    twin.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi], absolute=True)
        else:
            from oracle.oracle import JavaError
            try:
                exp = ora.processWatermark(step[1])
                scale = twin.processWatermark(step[1]) if twin is not None else None
            except JavaError:
                # a key's SessionContext is empty: activeWindows.get(0) throws in the reference
                # (SessionWindow.java:107), which ends a Flink job; the product reports the same exception
                with pytest.raises(pkg.ScottyError) as ei:
                    gpu.processWatermark(step[1])
                assert ei.value.code == -5  # SCOTTY_ERR_INDEX
                return total
            rows = gpu.processWatermark(step[1])
            total += same_keyed_windows(rows, exp, f64_cols=f64_cols, scale=scale)
            assert gpu.droppedCount() == ora.failed
    assert gpu.keyCount() == len(ora.ops)
    return total


@pytest.mark.parametrize("seed", range(16))
def test_keyed_streams_match_per_key_oracles(pkg, seed):
    rng = np.random.default_rng(5300 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    nkeys = int(rng.choice([1, 3, 50, 700, 5000]))
    if seed % 3 == 0:
        cfg = _session_cfg(rng, vt)
    else:
        wins = []
        for _ in range(int(rng.integers(1, 4))):
            r = rng.random()
            if r < 0.1:
                wins.append(FixedBand(Time, int(rng.integers(0, 3000)), int(rng.integers(1, 2000))))
            elif r < 0.5:
                wins.append(Tumbling(Time, _nz(int(rng.integers(5, 200)))))
            else:
                size = int(rng.integers(10, 300))
                wins.append(Sliding(Time, size, _nz(int(rng.integers(3, size + 1)))))
        cfg = dict(windows=wins, aggs=_aggs(rng, vt), lateness=int(rng.choice([1, 5, 100, 1000])))
    n = int(rng.integers(1000, 40_000))
    ts, vals = product().workloads.stream(n, [0.5, 2, 10][seed % 3], t0=int(rng.integers(0, 1000)),
                                          ooo_frac=[0.0, 0.2][seed % 2], max_delay=int(rng.integers(1, 200)),
                                          seed=seed, value_type=vt)
    keys = (rng.integers(0, nkeys, size=n) * 2654435761 % (2**32)).astype(np.uint32)
    sched = interval_schedule(ts, int(rng.integers(1, 6)), lag=int(rng.integers(0, 100)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a == SUM_F64]
    _keyed_run(pkg, cfg, keys, ts, vals, sched, vt=vt, f64_cols=f64_cols)


@pytest.mark.parametrize("seed", range(8))
def test_keyed_lane_path_equals_wavefront_replay(pkg, seed):
    """Context-free time windows on Eager slices run lane-per-key (keyed_lane.hip); the wavefront-per-key
    replay (exact_kernels.hip, tune "keyed_lane" 0) must leave the same rows -- larger streams and key counts
    than the oracle comparisons, out-of-order tuples, drops and slice GC."""
    rng = np.random.default_rng(6100 + seed)
    vt = ["i32", "i64", "f64", "i32"][seed % 4]
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]
    wins = [Sliding(Time, int(rng.integers(200, 3000)), _nz(int(rng.integers(20, 200)))),
            Tumbling(Time, _nz(int(rng.integers(30, 500))))][:1 + seed % 2]
    if seed % 3 == 1:
        wins.append(FixedBand(Time, int(rng.integers(0, 5000)), int(rng.integers(100, 5000))))
    aggs = _aggs(rng, vt)
    n = 300_000
    ts, vals = product().workloads.stream(n, [1, 4, 20][seed % 3], t0=int(rng.integers(0, 1000)),
                                          ooo_frac=[0.0, 0.3][seed % 2], max_delay=int(rng.integers(1, 400)),
                                          seed=seed, value_type=vt)
    nkeys = [10, 2_000, 30_000][seed % 3]
    keys = rng.integers(0, nkeys, size=n).astype(np.uint32)
    lateness = int(rng.choice([1, 50, 500]))
    ops = []
    f64_cols = [i for i, a in enumerate(aggs) if a == SUM_F64]
    for lane in (1, 0, 0)[:3 if f64_cols else 2]:  # f64: a third, |x|-fed replay operator gives sum |x| per row
        op = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
        op.tune("keyed_lane", lane)
        for a in aggs:
            op.addWindowFunction(a)
        op.setMaxLateness(lateness)
        for w in wins:
            op.addWindowAssigner(w)
        ops.append(op)
    sched = interval_schedule(ts, 12, lag=int(rng.integers(0, 300)), pushes_per_interval=2)
    total = 0
    for step in sched:
        if step[0] == "push":
            if step[2] > step[1]:
                for j, op in enumerate(ops):
                    v = vals[step[1]:step[2]]
                    op.processElements(keys[step[1]:step[2]], ts[step[1]:step[2]], np.abs(v) if j == 2 else v)
        else:
            a, b = ops[0].processWatermarkArrays(step[1]), ops[1].processWatermarkArrays(step[1])
            sc = ops[2].processWatermarkArrays(step[1]) if len(ops) == 3 else None
            total += same_keyed_arrays(a, b, f64_cols=f64_cols, scale=sc)
            assert ops[0].droppedCount() == ops[1].droppedCount()
    assert total > 0


def test_keyed_config4_reduced(pkg):
    """BASELINE configs[3] at reduced size: SlidingWindow(60 s, 1 s) SUM, keys Random(42).nextInt-like
    uniform over 20k keys, 90 s of event time, watermark every second."""
    n = 1_800_000
    ts, vals = product().workloads.stream(n, 20, t0=0, seed=42)
    keys = np.random.default_rng(42).integers(0, 20_000, size=n).astype(np.uint32)
    cfg = dict(windows=[Sliding(Time, 60_000, 1_000)], aggs=[SUM], lateness=1)
    sched = interval_schedule(ts, 90, lag=0)
    assert _keyed_run(pkg, cfg, keys, ts, vals, sched) > 20_000


def test_keyed_config4_full_size_per_key_totals(pkg):
    """C4 at the bench's full size: 2^26 tuples over 2^20 keys in one push (ts in [0, 1000) ms), SlidingWindow
    (60 s, 1 s), maxLateness 1.  At wm = 59999 every key's operator emits exactly [0, 60000) (SlidingWindow.
    triggerWindows, C/windowType/SlidingWindow.java:50-57: ws >= 0 and ws + size <= wm + 1), so its COUNT is
    the key's tuple count and its SUM the key's int32-wrapped value sum (SumAggregation.java:16-18)."""
    n, nk = 1 << 26, 1 << 20
    rng = np.random.default_rng(26)
    keys = rng.integers(0, nk, size=n, dtype=np.uint32)
    ts = np.arange(n, dtype=np.int64) // (n // 1000)
    vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    op = pkg.KeyedSlicingWindowOperator()
    op.addWindowFunction(SUM)
    op.addWindowFunction(COUNT)
    op.setMaxLateness(1)
    op.addWindowAssigner(Sliding(Time, 60_000, 1_000))
    op.processElements(keys, ts, vals)
    r = op.processWatermarkArrays(59_999)
    present = np.bincount(keys, minlength=nk)
    assert op.keyCount() == int((present > 0).sum())
    assert len(r["key"]) == op.keyCount()
    assert (r["start"] == 0).all() and (r["end"] == 60_000).all() and r["has_value"].all()
    k = r["key"].astype(np.int64)
    assert np.array_equal(np.sort(k), np.nonzero(present)[0])
    assert np.array_equal(r["values"][1], present[k])
    s = np.bincount(keys, weights=vals.astype(np.float64), minlength=nk)  # |sum| < 2^53: exact
    wrapped = ((s.astype(np.int64) + 2**31) % 2**32) - 2**31
    assert np.array_equal(r["values"][0], wrapped[k])


def test_keyed_large_batch_count_property(pkg):
    """2^24 tuples over 100k keys in one push: tumbling windows partition each key's in-order stream, so
    the COUNTs of all emitted windows add up to the tuple count."""
    n = 1 << 24
    rng = np.random.default_rng(8)
    keys = rng.integers(0, 100_000, size=n).astype(np.uint32)
    ts = np.arange(n, dtype=np.int64) // 1000
    vals = rng.integers(-100, 100, size=n).astype(np.int32)
    op = pkg.KeyedSlicingWindowOperator()
    op.addWindowFunction(COUNT)
    op.addWindowFunction(SUM)
    op.addWindowAssigner(Tumbling(Time, 1001))
    op.setMaxLateness(30_000)  # first watermark emits from max(0, wm - maxLateness) = 0 (WindowManager.java:43-44)
    op.processElements(keys, ts, vals)
    rows = op.processWatermark(int(ts.max()) + 2000)
    assert op.keyCount() == len(np.unique(keys))
    assert sum(w.getAggValues()[0] for _, w in rows if w.hasValue()) == n
    assert sum(w.getAggValues()[1] for _, w in rows if w.hasValue()) == int(vals.astype(np.int64).sum())


def test_keyed_table_growth_on_many_new_keys(pkg):
    """One push bringing 3 M new keys (the key table is sized for the known keys + max(known, 2^20) new ones, so this
    push overflows it: the insert pass stops, the table doubles and the pass re-runs), then a push of the same keys
    again (lookups only on the grown table).  Every key: HashMap.put on first sight (KeyedScottyWindowOperator.java:
    56-62), its tuples counted once per push; keys 0 and 0xFFFFFFFF among them."""
    n = 3 << 20
    rng = np.random.default_rng(31)
    keys = ((np.arange(1, n + 1, dtype=np.uint64) * 2654435761) % (1 << 32)).astype(np.uint32)  # distinct
    keys[0], keys[1] = 0xFFFFFFFF, 0  # the ends of the key range (0xFFFFFFFF once wrapped to the empty tag)
    assert len(np.unique(keys)) == n
    keys = rng.permutation(keys)
    vals = rng.integers(-1000, 1000, size=n).astype(np.int32)
    op = pkg.KeyedSlicingWindowOperator()
    op.addWindowFunction(COUNT)
    op.addWindowFunction(SUM)
    op.addWindowAssigner(Tumbling(Time, 1001))
    op.setMaxLateness(30_000)
    for step in range(2):
        ts = np.full(n, 10 + 1001 * step, dtype=np.int64)  # one tuple per key in tumbling window `step`
        op.processElements(keys, ts, vals)
        assert op.keyCount() == n
        r = op.processWatermarkArrays(1001 * step + 1500)  # triggers exactly that window
        assert len(r["start"]) == n and np.all(r["has_value"])
        assert np.all(r["values"][0] == 1)
        order = np.argsort(r["key"])
        assert np.array_equal(r["key"][order], np.sort(keys))
        assert np.array_equal(r["values"][1][order], vals[np.argsort(keys)].astype(np.int64))


def test_keyed_hash_sharding_equals_single_operator(pkg):
    """SURVEY §8(e) keyed: ranks own disjoint key sets (the router's key groups) and need no collective.  G=3
    keyed operators fed by KeyedShardRouter's split of one stream (each shard in arrival order) leave exactly the
    rows of one operator fed the whole stream."""
    rng = np.random.default_rng(77)
    n = 200_000
    ts, vals = product().workloads.stream(n, 4, t0=100, ooo_frac=0.2, max_delay=300, seed=77)
    keys = rng.integers(0, 5000, size=n).astype(np.uint32)
    wins = [Sliding(Time, 2000, 250), Tumbling(Time, 700)]

    def make():
        op = pkg.KeyedSlicingWindowOperator(device=0)
        op.addWindowFunction(SUM)
        op.addWindowFunction(MAX)
        op.setMaxLateness(500)
        for w in wins:
            op.addWindowAssigner(w)
        return op

    G = 3
    router = pkg.KeyedShardRouter(G)  # the product's host-side keyBy (scotty_route_keyed)
    whole, parts = make(), [make() for _ in range(G)]
    sched = interval_schedule(ts, 8, lag=400)
    total = 0
    for step in sched:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi <= lo:
                continue
            whole.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            for r, (k, t, v) in enumerate(router.route(keys[lo:hi], ts[lo:hi], vals[lo:hi])):
                if len(k):
                    parts[r].processElements(k, t, v)
        else:
            exp = {}
            for k, w in whole.processWatermark(step[1]):
                exp.setdefault(k, []).append(w)
            got = []
            for r in range(G):
                got += parts[r].processWatermark(step[1])
            total += same_keyed_windows(got, exp)
    assert sum(p.keyCount() for p in parts) == whole.keyCount()
    assert sum(p.droppedCount() for p in parts) == whole.droppedCount()
    assert total > 0


@pytest.mark.parametrize("seed", range(8))
def test_keyed_out_of_order_count_windows_match_per_key_oracles(pkg, seed):
    """Keyed operators with count windows on out-of-order streams: every key's operator keeps its own LazySlice
    record sets (per-key record arenas, grown on demand) -- KeyedScottyWindowOperator.java:56-86 per key."""
    rng = np.random.default_rng(9500 + seed)
    vt = ["i32", "i64", "i32", "f64"][seed % 4]
    wins = [Tumbling(Count, int(rng.integers(1, 20)))]
    if rng.random() < 0.5:
        size = int(rng.integers(2, 30))
        wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
    if rng.random() < 0.3:
        wins.append(Tumbling(Time, _nz(int(rng.integers(5, 100)))))
    cfg = dict(windows=wins, aggs=_lazy_aggs(rng, vt, invertible=seed % 4 == 1),
               lateness=int(rng.choice([10, 100, 1000])))
    nkeys = int(rng.choice([1, 7, 60, 400]))
    n = int(rng.integers(1000, 12_000))
    ts, vals = product().workloads.stream(n, [0.5, 2, 6][seed % 3], t0=int(rng.integers(0, 500)),
                                          ooo_frac=[0.05, 0.2][seed % 2], max_delay=int(rng.integers(1, 80)),
                                          seed=seed, value_type=vt)
    keys = (rng.integers(0, nkeys, size=n) * 2654435761 % (2**32)).astype(np.uint32)
    sched = interval_schedule(ts, int(rng.integers(1, 5)), lag=int(rng.integers(0, 60)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    f64_cols = [i for i, a in enumerate(cfg["aggs"]) if a & 0xFFFF == SUM_F64]
    _keyed_run(pkg, cfg, keys, ts, vals, sched, vt=vt, f64_cols=f64_cols)
