"""Host-buffer ingest (csrc/host_ingest.cpp): micro-batches handed over in host memory -- the op's pinned staging
slots (scotty_host_buffers, DMA'd in place) or pageable arrays (chunked through pinned staging on a copy stream) --
leave the oracle's windows on every engine (grid path, exact engine, keyed).  Every other parity test pushes
pageable numpy arrays and so runs the pageable path too; here: pinned slots, the multi-chunk pageable pipeline, and
slot alternation."""
import numpy as np
import pytest

from helpers import product, build_ops, same_windows, same_keyed_windows, KeyedOracle
from specs import Tumbling, Sliding, Session, Time, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return product()


def _push(op, mode, *cols):
    """cols: (ts, vals) or (keys, ts, vals) for keyed ops; pinned: through a freshly handed-out slot."""
    if mode == "pageable":
        op.processElements(*cols)
        return
    if len(cols) == 2:
        ts, vals = cols
        hts, hv = op.hostBuffers(len(ts))
        hts[:], hv[:] = ts, vals
        op.processElements(hts, hv)
    else:
        keys, ts, vals = cols
        hts, hv, hk = op.hostBuffers(len(ts))
        hts[:], hv[:], hk[:] = ts, vals, keys
        op.processElements(hk, hts, hv)


@pytest.mark.parametrize("mode", ["pinned", "pageable"])
def test_grid_path_host_pushes_match_oracle(pkg, mode):
    """Grid path (context-free time windows): 4 watermark intervals, two pushes each; the last interval's second
    push is 5M tuples -- past the 4M-tuple chunk of the pageable pipeline."""
    rng = np.random.default_rng(11)
    wins = [Tumbling(Time, int(s)) for s in rng.integers(200, 3000, size=12)] + [Sliding(Time, 2000, 300)]
    gpu, ora = build_ops(dict(windows=wins, aggs=[SUM, COUNT], lateness=1))
    t0 = 0
    for step in range(4):
        n = 5_600_000 if step == 3 else 600_000
        ts = t0 + np.arange(n, dtype=np.int64) // 1000
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
        for lo, hi in ((0, n // 8), (n // 8, n)):
            _push(gpu, mode, ts[lo:hi], vals[lo:hi])
            ora.processElements(ts[lo:hi], vals[lo:hi])
        wm = int(ts[-1])
        same_windows(gpu.processWatermark(wm), ora.processWatermark(wm))
        t0 = wm + 1


@pytest.mark.parametrize("mode", ["pinned", "pageable"])
def test_exact_engine_host_pushes_match_oracle(pkg, mode):
    """Session + sliding windows, 20% out-of-order: the exact engine's batch path from host memory."""
    wins = [Sliding(Time, 3000, 500), Session(Time, 300)]
    gpu, ora = build_ops(dict(windows=wins, aggs=[MIN, MAX], lateness=1000))
    ts, vals = product().workloads.stream(200_000, 20, t0=0, ooo_frac=0.2, max_delay=300, seed=12,
                                          gaps=[(i, 1500) for i in range(50_000, 200_000, 50_000)])
    for lo in range(0, len(ts), 50_000):
        hi = lo + 50_000
        _push(gpu, mode, ts[lo:hi], vals[lo:hi])
        ora.processElements(ts[lo:hi], vals[lo:hi])
        wm = int(ts[:hi].max()) - 300
        same_windows(gpu.processWatermark(wm), ora.processWatermark(wm))


@pytest.mark.parametrize("mode", ["pinned", "pageable"])
def test_keyed_host_pushes_match_per_key_oracles(pkg, mode):
    rng = np.random.default_rng(13)
    cfg = dict(windows=[Sliding(Time, 5000, 1000)], aggs=[SUM, COUNT], lateness=1)
    gpu = pkg.KeyedSlicingWindowOperator(device=0)
    for a in cfg["aggs"]:
        gpu.addWindowFunction(a)
    gpu.setMaxLateness(1)
    for w in cfg["windows"]:
        gpu.addWindowAssigner(w)
    ora = KeyedOracle(cfg)
    for step in range(4):
        n = 20_000
        ts = step * 1000 + np.arange(n, dtype=np.int64) // 20
        vals = rng.integers(-1000, 1000, size=n).astype(np.int32)
        keys = rng.integers(0, 300, size=n).astype(np.uint32)
        _push(gpu, mode, keys, ts, vals)
        ora.processElements(keys, ts, vals)
        wm = int(ts[-1])
        same_keyed_windows(gpu.processWatermark(wm), ora.processWatermark(wm))
    assert gpu.keyCount() == len(ora.ops)


def test_pinned_slots_alternate_and_pageable_path_equal(pkg):
    """Two slots alternate (the third request returns the first slot once its DMA is done); six pushes filled while
    the other slot is in flight leave the windows of the same six pushes from pageable arrays (8M tuples each: two
    chunks of the pageable pipeline)."""
    wins = [Tumbling(Time, 100), Sliding(Time, 700, 100)]
    pin, pag = build_ops(dict(windows=wins, aggs=[SUM, COUNT], lateness=1))[0], \
        build_ops(dict(windows=wins, aggs=[SUM, COUNT], lateness=1))[0]
    addrs = []
    for step in range(6):
        n = 8_000_000
        ts = step * 1000 + np.arange(n, dtype=np.int64) // 8000
        vals = np.full(n, step + 1, dtype=np.int32)
        hts, hv = pin.hostBuffers(n)
        addrs.append(hts.ctypes.data)
        hts[:], hv[:] = ts, vals
        pin.processElements(hts, hv)
        pag.processElements(ts, vals)
    assert addrs[0] == addrs[2] == addrs[4] and addrs[1] == addrs[3] and addrs[0] != addrs[1]
    a, b = pin.processWatermark(5999), pag.processWatermark(5999)
    assert len(a) > 0
    same_windows(a, b)
    assert pin.processedCount() == pag.processedCount() == 6 * 8_000_000
