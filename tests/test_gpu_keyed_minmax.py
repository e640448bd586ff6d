"""Keyed MIN / MAX window assembly from block summaries (north_star: "a sparse table for non-invertible
ones such as min and max"): the key-interleaved store keeps, per block of XK_MB = 16 slice positions, in-block
prefix and suffix minima / maxima (exact_common.h XK_QN...), and the lane watermark kernel assembles a window of
positions [lo, hi) from SN[lo], one prefix word per whole block and QN[hi - 1] (keyed_lane.hip, lane_wm_emit_kernel)
instead of LazyAggregateStore.aggregate's scan of every contained slice (S/aggregationstore/LazyAggregateStore.java:
83-111).  Checked against one oracle operator per key (the connector's HashMap, F/KeyedScottyWindowOperator.java:
56-86) and against the wavefront-per-key replay with its per-slice scan (tune "keyed_lane" 0): windows spanning one
block, several blocks and many, in-order and out-of-order streams (late tuples change older slices and so the
summaries of old blocks), slice compaction, int32 and int64 values."""
import numpy as np
import pytest

from helpers import product, KeyedOracle, same_keyed_windows, interval_schedule
from specs import Tumbling, Sliding, FixedBand, Time, SUM, COUNT, MIN, MAX, SUM_I64, MIN_I64, MAX_I64

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return product()


def _run(pkg, cfg, keys, ts, vals, sched, vt="i32", ab=True):
    """Product (lane path, key-interleaved store) vs per-key oracles and vs the wavefront replay (keyed_lane 0)."""
    vtc = {"i32": pkg.VALUE_I32, "i64": pkg.VALUE_I64}[vt]
    ops = []
    for lane in ((1, 0) if ab else (1,)):
        op = pkg.KeyedSlicingWindowOperator(device=0, value_type=vtc)
        op.tune("keyed_lane", lane)
        for a in cfg["aggs"]:
            op.addWindowFunction(a)
        op.setMaxLateness(cfg["lateness"])
        for w in cfg["windows"]:
            op.addWindowAssigner(w)
        ops.append(op)
    ora = KeyedOracle(cfg)
    total = 0
    for step in sched:
        if step[0] == "push":
            lo, hi = step[1], step[2]
            if hi <= lo:
                continue
            for op in ops:
                op.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            ora.processElements(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        else:
            exp = ora.processWatermark(step[1])
            for op in ops:
                total += same_keyed_windows(op.processWatermark(step[1]), exp)
                assert op.droppedCount() == ora.failed
    return total // len(ops)


@pytest.mark.parametrize("seed", range(8))
def test_keyed_min_max_blocks_match_oracle(pkg, seed):
    rng = np.random.default_rng(7700 + seed)
    vt = ["i32", "i64"][seed % 2]
    aggs = {"i32": [MIN, MAX, SUM, COUNT], "i64": [MAX_I64, COUNT, MIN_I64, SUM_I64]}[vt]
    aggs = aggs[:2 + seed % 3]
    # slides of 7-40 ms under windows of 40x-70x the slide: one window spans 3-5 summary blocks; a short tumbling
    # window beside it keeps within-block windows in the mix
    slide = int(rng.integers(7, 41))
    slide += 1 if slide & (slide - 1) == 0 else 0
    wins = [Sliding(Time, slide * int(rng.integers(40, 71)), slide)]
    if seed % 3 == 0:
        wins.append(Tumbling(Time, 3 * slide + 1))
    if seed % 4 == 1:
        wins.append(FixedBand(Time, int(rng.integers(0, 2000)), int(rng.integers(500, 4000))))
    cfg = dict(windows=wins, aggs=aggs, lateness=int(rng.choice([1, 50, 400])))
    n = int(rng.integers(20_000, 60_000))
    ts, vals = product().workloads.stream(n, [0.5, 1, 3][seed % 3], t0=int(rng.integers(0, 500)),
                                          ooo_frac=[0.0, 0.15][seed % 2], max_delay=int(rng.integers(1, 300)),
                                          seed=seed, value_type=vt)
    nkeys = int(rng.choice([1, 5, 60, 900]))
    keys = rng.integers(0, nkeys, size=n).astype(np.uint32)
    sched = interval_schedule(ts, int(rng.integers(4, 14)), lag=int(rng.integers(0, 150)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    assert _run(pkg, cfg, keys, ts, vals, sched, vt) > 0


def test_keyed_min_max_long_windows_and_compaction(pkg):
    """Windows over ~250 slices (15 whole blocks) of a few keys, a stream long enough that each key's slice store is
    compacted to the front (positions move: every summary is rebuilt), with late tuples into old blocks."""
    n = 400_000
    ts, vals = product().workloads.stream(n, 2, t0=0, ooo_frac=0.05, max_delay=200, seed=5)
    keys = np.random.default_rng(5).integers(0, 3, size=n).astype(np.uint32)
    cfg = dict(windows=[Sliding(Time, 2503, 10)], aggs=[MIN, MAX, COUNT], lateness=300)
    sched = interval_schedule(ts, 40, lag=250)
    assert _run(pkg, cfg, keys, ts, vals, sched, ab=False) > 10_000


def test_keyed_config4_min_max_reduced(pkg):
    """C4's stream shape with MIN_I32 + MAX_I32 (the verdict's keyed min/max case) at reduced size: SlidingWindow(60 s,
    1 s) over 20k uniform keys, 90 s of event time, a watermark per second: each window covers 60 slices (4 blocks)."""
    n = 1_800_000
    ts, vals = product().workloads.stream(n, 20, t0=0, seed=42)
    keys = np.random.default_rng(42).integers(0, 20_000, size=n).astype(np.uint32)
    cfg = dict(windows=[Sliding(Time, 60_000, 1_000)], aggs=[MIN, MAX], lateness=1)
    sched = interval_schedule(ts, 90, lag=0)
    assert _run(pkg, cfg, keys, ts, vals, sched, ab=False) > 20_000
