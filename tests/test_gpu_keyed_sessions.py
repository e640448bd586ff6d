"""Keyed session windows at scale: KeyedScottyWindowOperator with SessionWindow + SlidingWindow per key
(flink-connector/.../KeyedScottyWindowOperator.java:56-86 over C/windowType/SessionWindow.java:40-116), 2^17 keys,
20 % out-of-order tuples, streams that pause so every key's session closes -- the wavefront-per-key replay
(exact_kernels.hip replay_kernel) at a key count two orders of magnitude above the other keyed parity tests.

The per-key oracle runs on a random sample of the keys (each sampled key's tuples in arrival order, the connector's
HashMap semantics: one independent operator per key), and the product's rows of exactly those keys must match it
bit-exactly at every watermark; the other keys' rows are checked for their count and ordering invariants."""
import numpy as np
import pytest

from helpers import product, KeyedOracle, same_keyed_windows
from specs import Sliding, Session, Time, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu


def _stream(step, B, nkeys, rng, period=5, silence=2000, max_delay=500, late_frac=0.2):
    t_begin = 1000 + step * 1000 + (step // period) * silence
    keys = rng.integers(0, nkeys, B).astype(np.uint32)
    ts = t_begin + np.arange(B, dtype=np.int64) * 1000 // B
    late = rng.random(B) < late_frac
    ts = np.where(late, ts - rng.integers(1, max_delay + 1, B), ts)
    vals = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    return keys, ts, vals, t_begin + 999 - max_delay


def _rows_of(arrs, sample):
    """(key, AggregateWindow) rows of the sampled keys, in the product's order."""
    pkg = product()
    sel = np.flatnonzero(np.isin(arrs["key"], sample))
    out = []
    for i in sel:
        has = bool(arrs["has_value"][i])
        vals = [int(c[i]) for c in arrs["values"]] if has else []
        out.append((int(arrs["key"][i]), pkg.AggregateWindow(int(arrs["start"][i]), int(arrs["end"][i]),
                                                             int(arrs["measure"][i]), has, vals)))
    return out


@pytest.mark.parametrize("nkeys,B", [(1 << 17, 1 << 21)])
def test_keyed_sessions_at_scale_match_sampled_oracles(nkeys, B):
    pkg = product()
    cfg = dict(windows=[Sliding(Time, 10_000, 1000), Session(Time, 1000)], aggs=[SUM, COUNT, MIN, MAX], lateness=1000)
    op = pkg.KeyedSlicingWindowOperator(device=0)
    for a in cfg["aggs"]:
        op.addWindowFunction(a)
    op.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        op.addWindowAssigner(w)
    rng = np.random.default_rng(2024)
    sample = np.sort(rng.choice(nkeys, 1500, replace=False)).astype(np.uint32)
    ora = KeyedOracle(cfg)
    total = checked = sessions = 0
    for step in range(12):
        keys, ts, vals, wm = _stream(step, B, nkeys, rng)
        op.processElements(keys, ts, vals)
        m = np.isin(keys, sample)
        ora.processElements(keys[m], ts[m], vals[m])
        arrs = op.processWatermarkArrays(wm)
        n = len(arrs["start"])
        total += n
        # every row is well formed: start < end, a key's rows contiguous (the connector loops over its keys)
        assert np.all(arrs["start"] < arrs["end"])
        if n:
            k = arrs["key"]
            changes = np.count_nonzero(k[1:] != k[:-1]) + 1
            assert changes == len(np.unique(k))
        sessions += int(np.count_nonzero(arrs["end"] - arrs["start"] != 10_000))
        checked += same_keyed_windows(_rows_of(arrs, sample), ora.processWatermark(wm))
    assert op.keyCount() == nkeys
    assert checked > 1500 and sessions > nkeys  # every key's session closed at each pause
    print("rows %d, sampled rows checked %d, session rows %d" % (total, checked, sessions))


def _nz(x):  # a power-of-two size / slide makes the reference loop forever
    return x + 1 if x & (x - 1) == 0 else x


@pytest.mark.parametrize("seed", range(16))
def test_lane_session_kernel_equals_wavefront_replay(seed):
    """The lane-per-key session replay (keyed_lane_session.hip, the default for keyed session windows) against the
    wavefront replay (scotty_tune "keyed_lane_session" 0, exact_kernels.hip) on random keyed streams: one or two
    session windows (gaps 20-800 ms) beside 0-2 context-free windows, out-of-order shares 0-50 % with delays up to 2 gaps
    (shiftStart / split / merge / new-session-before edits), pauses that close sessions, i32 / i64 / f64 values.
    Seeds 12-15 shift the stream below zero (negative event times: fixed edges crossed without an append still
    advance the pending edge, S/StreamSlicer.java:65-69), seeds 12 and 14 register session windows only (no fixed
    edge at all: the fast path's has_fixed == 0 case).
    Every watermark's rows (bounds, hasValue, values; f64 sums within the f64 bound) and the dropped counts match."""
    from specs import Tumbling, SUM_I64, MIN_I64, MAX_I64, SUM_F64, MIN_F64, MAX_F64
    pkg = product()
    rng = np.random.default_rng(6100 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    aggs = [x for x in aggs if rng.random() < 0.7] or [aggs[0]]
    gaps = [int(rng.integers(20, 800)) for _ in range(1 + (seed % 3 == 2))]
    wins = [Session(Time, g) for g in gaps]
    for _ in range(0 if seed in (12, 14) else int(rng.integers(1 if seed >= 12 else 0, 3))):
        if rng.random() < 0.5:
            wins.append(Tumbling(Time, _nz(int(rng.integers(50, 2000)))))
        else:
            size = int(rng.integers(100, 3000))
            wins.append(Sliding(Time, size, _nz(int(rng.integers(20, size + 1)))))
    rng.shuffle(wins)
    lateness = int(rng.choice([1, 50, 1000, 5000]))
    nkeys = int(rng.choice([7, 300, 5000, 40_000]))
    n = int(rng.integers(50_000, 400_000))
    rate = [0.5, 2, 10, 40][seed % 4]
    pauses = [(int(i), int(rng.integers(1, 4)) * max(gaps)) for i in range(int(rng.integers(5000, 40_000)), n, 50_000)]
    ts, vals = pkg.workloads.stream(n, rate, t0=int(rng.integers(0, 2000)), ooo_frac=float(rng.choice([0, 0.05, 0.2, 0.5])),
                                    max_delay=int(rng.integers(1, 2 * max(gaps) + 2)), seed=seed, value_type=vt,
                                    gaps=pauses)
    keys = ((rng.integers(0, nkeys, size=n) * 2654435761) % (1 << 32)).astype(np.uint32)
    if seed >= 12:  # the stream starts below zero and crosses it
        ts = ts - int(rng.integers(2000, 30_000))
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]

    def make(lane):
        op = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
        op.tune("keyed_lane_session", (1 + seed % 2) if lane else 0)  # odd seeds: the kernel's 3-waves build
        for x in aggs:
            op.addWindowFunction(x)
        op.setMaxLateness(lateness)
        for w in wins:
            op.addWindowAssigner(w)
        return op
    lane, wave = make(True), make(False)
    f64_cols = [i for i, x in enumerate(aggs) if x == SUM_F64]
    twin = make(False) if f64_cols else None  # |x|-fed replay: sum |x| per row (helpers.F64_REL)
    total = errors = 0
    from helpers import interval_schedule, same_keyed_arrays
    for step in interval_schedule(ts, int(rng.integers(3, 12)), lag=int(rng.integers(0, 2 * max(gaps))),
                                  pushes_per_interval=int(rng.integers(1, 3))):
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                lane.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                wave.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                if twin is not None:
                    twin.processElements(keys[lo:hi], ts[lo:hi], np.abs(vals[lo:hi]))
        else:
            sc = None
            try:
                if twin is not None:
                    try:
                        sc = twin.processWatermarkArrays(step[1])
                    except pkg.ScottyError:
                        pass  # the same throw as the wavefront replay's below (same timestamps)
                exp = wave.processWatermarkArrays(step[1])
            except pkg.ScottyError as e:
                # SessionWindow.triggerWindows reads getWindow(0) of a key whose sessions all closed at an earlier
                # watermark (SessionWindow.java:107-116): the reference throws out of the connector's key loop.  Both
                # kernels leave the same state behind, so the lane path must throw the same way
                assert e.code == -5
                with pytest.raises(pkg.ScottyError) as ei:
                    lane.processWatermarkArrays(step[1])
                assert ei.value.code == -5
                errors += 1
                continue
            total += same_keyed_arrays(lane.processWatermarkArrays(step[1]), exp, f64_cols=f64_cols, scale=sc)
            assert lane.droppedCount() == wave.droppedCount()
    assert lane.keyCount() == wave.keyCount()
    assert total > 0 or errors > 0


@pytest.mark.parametrize("seed", range(8))
def test_packed_replay_records_equal_16_byte_records(seed):
    """An int32 keyed batch whose key bits plus the bits of its event-time span fit one 32-bit word is sorted and
    replayed as packed 8-byte records {key << tb | ts - tbase, value} (keyed_kernels.hip Rec<8>); scotty_tune
    "keyed_pack_records" 0 keeps the 16-byte records.  Dense key ranges of 3-20 bits, batches spanning a few ms to
    minutes (some fit, some do not), timestamps offset up to 2^40: every watermark's rows and the dropped counts
    match, and the packed layout is taken where it fits (debug stat 107: the last replay's record bytes)."""
    pkg = product()
    rng = np.random.default_rng(7300 + seed)
    gap = int(rng.integers(20, 800))
    wins = [Session(Time, gap)]
    if seed % 2:
        wins.append(Sliding(Time, 2000, 300 + seed))
    aggs = [SUM, COUNT, MIN, MAX]
    nkeys = [7, 300, 5000, 1 << 20][seed % 4]
    n = int(rng.integers(100_000, 400_000))
    rate = [0.5, 2, 10, 40][(seed // 2) % 4]
    t0 = [0, 1 << 40][seed % 2] + int(rng.integers(0, 2000))
    pauses = [(int(i), int(rng.integers(1, 4)) * gap) for i in range(int(rng.integers(5000, 40_000)), n, 50_000)]
    ts, vals = pkg.workloads.stream(n, rate, t0=t0, ooo_frac=float(rng.choice([0.05, 0.2, 0.5])),
                                    max_delay=int(rng.integers(1, 2 * gap + 2)), seed=seed, value_type="i32",
                                    gaps=pauses)
    keys = rng.integers(0, nkeys, size=n).astype(np.uint32)
    lateness = int(rng.choice([50, 1000]))

    def make(pack):
        op = pkg.KeyedSlicingWindowOperator(device=0)
        op.tune("keyed_pack_records", pack)
        for x in aggs:
            op.addWindowFunction(x)
        op.setMaxLateness(lateness)
        for w in wins:
            op.addWindowAssigner(w)
        return op
    packed, plain = make(1), make(0)
    from helpers import interval_schedule, same_keyed_arrays
    total, errors, layouts = 0, 0, set()
    for step in interval_schedule(ts, int(rng.integers(3, 12)), lag=int(rng.integers(0, 2 * gap)),
                                  pushes_per_interval=int(rng.integers(1, 3))):
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                packed.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                plain.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                layouts.add(packed._debug_stat(107))
                assert plain._debug_stat(107) == 16
        else:
            try:
                exp = plain.processWatermarkArrays(step[1])
            except pkg.ScottyError as e:  # the reference's throw out of the key loop (see the test above): both alike
                with pytest.raises(pkg.ScottyError) as ei:
                    packed.processWatermarkArrays(step[1])
                assert ei.value.code == e.code
                errors += 1
                continue
            total += same_keyed_arrays(packed.processWatermarkArrays(step[1]), exp)
            assert packed.droppedCount() == plain.droppedCount()
    assert packed.keyCount() == plain.keyCount()
    assert total > 0 or errors > 0
    if nkeys <= 5000:
        assert 8 in layouts


@pytest.mark.parametrize("seed", range(6))
def test_ten_bit_digit_sort_equals_eight_bit_sort(seed):
    """The keyed replay's stable sort by key (keyed_kernels.hip): scotty_tune "keyed_sort_digit10" 1 sorts 17-20-bit keys
    in two 10-bit digit passes (measured slower, so the default keeps three 8-bit ones, 0).  A
    stable sort has one result, so
    every watermark's rows and the dropped counts must be identical; session and count windows (lane-session kernel,
    wavefront replay), packed 8-byte and 16-byte records, key ranges from 2^16 + 1 to 2^20."""
    from specs import Tumbling, Count
    pkg = product()
    rng = np.random.default_rng(8800 + seed)
    nkeys = [(1 << 16) + 7, 1 << 18, 1 << 20, 700_001, 1 << 17, (1 << 20) - 3][seed]
    wins = [Session(Time, int(rng.integers(50, 500))), Sliding(Time, 2000, 250)] if seed % 2 == 0 else \
        [Tumbling(Count, int(rng.integers(3, 30))), Sliding(Time, 1500, 300)]
    n = 600_000
    ts, vals = pkg.workloads.stream(n, [20, 200][seed % 2], t0=int(rng.integers(0, 3000)), ooo_frac=0.2,
                                    max_delay=400, seed=seed, value_type="i32")
    keys = rng.integers(0, nkeys, size=n).astype(np.uint32)

    def make(d10, pack):
        op = pkg.KeyedSlicingWindowOperator(device=0)
        op.tune("keyed_sort_digit10", d10)
        op.tune("keyed_pack_records", pack)
        for x in (SUM, COUNT, MIN, MAX):
            op.addWindowFunction(x)
        op.setMaxLateness(1000)
        for w in wins:
            op.addWindowAssigner(w)
        return op
    pack = seed % 3 != 2
    a, b = make(1, pack), make(0, pack)
    from helpers import interval_schedule, same_keyed_arrays
    total = 0
    for step in interval_schedule(ts, 6, lag=300, pushes_per_interval=2):
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi > lo:
                a.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                b.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        else:
            try:
                exp = b.processWatermarkArrays(step[1])
            except pkg.ScottyError as e:
                with pytest.raises(pkg.ScottyError) as ei:
                    a.processWatermarkArrays(step[1])
                assert ei.value.code == e.code
                continue
            total += same_keyed_arrays(a.processWatermarkArrays(step[1]), exp)
            assert a.droppedCount() == b.droppedCount()
    assert a.keyCount() == b.keyCount()
    assert total > 0
