"""Deterministic sharded-run cases shared by the worker ranks and the checking test (no GPU needed here)."""
import numpy as np

from helpers import product, interval_schedule
from specs import Tumbling, Sliding, FixedBand, Time, Count, SUM, COUNT, MIN, MAX


def case(cid):
    rng = np.random.default_rng(600 + cid)
    wl = product().workloads
    if cid == 0:   # C2-like: many tumbling windows, in-order
        sizes = wl.random_tumbling_sizes(200, 1, 20, seed=10)
        cfg = dict(windows=[Tumbling(Time, s) for s in sizes], aggs=[SUM, COUNT], lateness=1)
        ts, vals = wl.stream(400_000, 20, t0=0, seed=cid)
    elif cid == 1:  # sliding + tumbling, 20 % out-of-order across chunk boundaries
        cfg = dict(windows=[Sliding(Time, 3000, 61), Tumbling(Time, 997)], aggs=[SUM, COUNT, MIN, MAX], lateness=800)
        ts, vals = wl.stream(300_000, 25, t0=100, ooo_frac=0.2, max_delay=500, seed=cid)
    elif cid == 3:  # sparse: tuples jump over grid points by more than maxLateness at chunk cuts
        cfg = dict(windows=[Tumbling(Time, 5), Sliding(Time, 40, 7)], aggs=[SUM, COUNT], lateness=2)
        ts, vals = wl.stream(6000, 0.25, t0=1000, ooo_frac=0.1, max_delay=3, seed=cid)
        ts = ts + np.cumsum(rng.integers(0, 4, size=len(ts)))
        sched = interval_schedule(ts, 40, lag=5, pushes_per_interval=3)
        return cfg, ts, vals, sched
    elif cid == 4:  # C5-like: randomCount count windows, in-order with ties, a few too-late tuples (dropped)
        sizes = wl.random_count_sizes(50, 100, 5000, seed=10)
        cfg = dict(windows=[Tumbling(Count, s) for s in sizes], aggs=[SUM, COUNT, MIN, MAX], lateness=1)
        n = 300_000
        ts = 50 + np.arange(n, dtype=np.int64) // 30
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
        late = rng.choice(np.arange(n // 3, n), size=4, replace=False)
        ts[late] = 10
        sched = interval_schedule(ts, 7, lag=0, pushes_per_interval=2)
        return cfg, ts, vals, sched
    elif cid == 5:  # dense count edges (every few tuples): cells straddle chunk cuts, edge-heavy steps
        cfg = dict(windows=[Sliding(Count, 9, 4), Tumbling(Count, 7), FixedBand(Count, 1000, 30_000)],
                   aggs=[SUM, MAX], lateness=20)
        n = 60_000
        ts = 1000 + np.arange(n, dtype=np.int64) // 3
        vals = rng.integers(-1000, 1000, size=n, dtype=np.int64).astype(np.int32)
        sched = interval_schedule(ts, 9, lag=3, pushes_per_interval=3)
        return cfg, ts, vals, sched
    elif cid == 6:  # count + sliding time windows, in-order unique timestamps
        cfg = dict(windows=[Tumbling(Count, 1000), Sliding(Time, 60000, 1000)], aggs=[SUM, COUNT], lateness=1)
        n = 200_000
        ts = 5 + np.cumsum(rng.integers(1, 4, size=n)).astype(np.int64)
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
        sched = interval_schedule(ts, 80, lag=0, pushes_per_interval=2)
        return cfg, ts, vals, sched
    elif cid == 7:  # count + time windows with ties, lateness > slide, tiny pushes (empty chunks on a rank)
        cfg = dict(windows=[Sliding(Time, 50, 7), Tumbling(Count, 13), Tumbling(Time, 11), FixedBand(Count, 100, 900)],
                   aggs=[SUM, COUNT, MIN], lateness=30)
        n = 20_000
        ts = 3000 + np.sort(rng.integers(0, 6000, size=n)).astype(np.int64)
        vals = rng.integers(-1000, 1000, size=n, dtype=np.int64).astype(np.int32)
        sched = []
        lo = 0
        for size in [1, 1, 3, 2, 50, 1, 400] + [997] * 19 + [n]:
            hi = min(n, lo + size)
            if hi > lo:
                sched += [("push", lo, hi), ("wm", int(ts[hi - 1]) - 2)]
            lo = hi
        return cfg, ts, vals, sched
    else:           # lateness edge skipping on jumps + fixed band
        cfg = dict(windows=[Tumbling(Time, 13), FixedBand(Time, 5000, 2000)], aggs=[SUM, MAX], lateness=3)
        ts, vals = wl.stream(120_000, 2, t0=7, ooo_frac=0.05, max_delay=2, seed=cid,
                             gaps=[(i, int(rng.integers(50, 900))) for i in range(5000, 120_000, 7000)])
    sched = interval_schedule(ts, 6, lag=50 if cid != 1 else 500, pushes_per_interval=2)
    return cfg, ts, vals, sched
