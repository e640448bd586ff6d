"""The lane-per-key replay of keyed LazySlice record sets (keyed_lane_count.hip, the default for keyed count windows
without session windows) against the wavefront replay (scotty_tune "keyed_lane_count" 0, exact_kernels.hip
replay_kernel), which is itself pinned by the per-key oracles (tests/test_gpu_exact.py, tests/test_gpu_keyed_count.py).

Random keyed streams: tumbling or sliding count windows (S/SliceManager.java:64-87's count-shift loop for every
out-of-order tuple), optionally beside tumbling / sliding time windows, out-of-order shares 0-50 %, lateness 1-5000,
i32 / i64 / f64 values, SUM / COUNT / MIN / MAX, duplicate timestamps (TreeSet dedupe, S/slice/StreamRecord.java:25-27),
key counts 7-2000, small slice / record capacities so the host grows them between retries and the arena compacts.
Every watermark's rows (bounds, hasValue, values; f64 sums within the f64 bound against an |x|-fed twin) and the
dropped counts match; a watermark that throws (LazyAggregateStore.aggregate's getSlice(-1) once a count window's
start slice is gone) throws on both."""
import numpy as np
import pytest

from helpers import product, interval_schedule, same_keyed_arrays
from specs import Tumbling, Sliding, Time, Count, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu


def _nz(x):  # a power-of-two time size / slide makes the reference loop forever
    return x + 1 if x & (x - 1) == 0 else x


@pytest.mark.parametrize("seed", range(12))
def test_lane_count_kernel_equals_wavefront_replay(seed):
    from specs import SUM_I64, MIN_I64, MAX_I64, SUM_F64, MIN_F64, MAX_F64
    pkg = product()
    rng = np.random.default_rng(7300 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    aggs = {"i32": [SUM, COUNT, MIN, MAX], "i64": [SUM_I64, COUNT, MIN_I64, MAX_I64],
            "f64": [SUM_F64, COUNT, MIN_F64, MAX_F64]}[vt]
    aggs = [x for x in aggs if rng.random() < 0.7] or [aggs[0]]
    csize = int(rng.integers(3, 60))
    wins = [Tumbling(Count, csize) if rng.random() < 0.6 else Sliding(Count, csize, int(rng.integers(1, csize + 1)))]
    for _ in range(int(rng.integers(0, 3))):
        if rng.random() < 0.5:
            wins.append(Tumbling(Time, _nz(int(rng.integers(50, 2000)))))
        else:
            size = int(rng.integers(100, 3000))
            wins.append(Sliding(Time, size, _nz(int(rng.integers(20, size + 1)))))
    rng.shuffle(wins)
    lateness = int(rng.choice([1, 50, 1000, 5000]))
    nkeys = int(rng.choice([7, 300, 2000]))  # >= 50 tuples per key: count windows fire
    n = int(rng.integers(100_000, 300_000))
    rate = [0.5, 2, 10, 40][seed % 4]
    ts, vals = pkg.workloads.stream(n, rate, t0=int(rng.integers(0, 2000)), ooo_frac=float(rng.choice([0, 0.05, 0.2, 0.5])),
                                    max_delay=int(rng.integers(1, 600)), seed=seed, value_type=vt)
    if seed % 3 == 1:  # coarse timestamps: many duplicates per key (TreeSet.add drops an equal-ts record)
        ts = ts // 7 * 7
    keys = ((rng.integers(0, nkeys, size=n) * 2654435761) % (1 << 32)).astype(np.uint32)
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64, "f64": pkg.VALUE_F64}[vt]

    def make(lane):
        op = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
        op.tune("keyed_lane_count", 1 if lane else 0)
        if seed % 2 == 0:  # small capacities: retries that grow them, arena compactions
            op.tune("slice_capacity", 16)
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
    for step in interval_schedule(ts, int(rng.integers(3, 12)), lag=int(rng.integers(0, 800)),
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
                        pass  # the same throw as the wavefront replay's below
                exp = wave.processWatermarkArrays(step[1])
            except pkg.ScottyError as e:
                with pytest.raises(pkg.ScottyError) as ei:
                    lane.processWatermarkArrays(step[1])
                assert ei.value.code == e.code
                errors += 1
                continue
            total += same_keyed_arrays(lane.processWatermarkArrays(step[1]), exp, f64_cols=f64_cols, scale=sc)
            assert lane.droppedCount() == wave.droppedCount()
    assert lane.keyCount() == wave.keyCount()
    assert total > 0 or errors > 0
    print("rows %d, throwing watermarks %d" % (total, errors))
