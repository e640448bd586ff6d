"""Keyed out-of-order count windows at scale: KeyedScottyWindowOperator (flink-connector/.../
KeyedScottyWindowOperator.java:56-86) with TumblingWindow(Count) + SlidingWindow(Time) per key, 2^17 keys, 20 %
out-of-order tuples.  Count windows make every slice a LazySlice with a TreeSet record set (S/slice/SliceFactory.java:
17-22, S/slice/LazySlice.java) and every out-of-order tuple runs SliceManager's count-shift loop (S/SliceManager.java:
64-87): the per-key replay path (exact_kernels.hip replay_kernel), here at a key count two orders of magnitude above
the other keyed count tests (tests/test_gpu_exact.py, <= 400 keys).

The per-key oracle runs on a random sample of the keys (their tuples in arrival order: one independent operator per
key, the connector's HashMap), and the product's rows of exactly those keys must match it bit-exactly at every
watermark; every row is checked for well-formedness."""
import numpy as np
import pytest

from helpers import product, KeyedOracle, same_keyed_windows
from specs import Sliding, Tumbling, Time, Count, SUM, COUNT, MIN, MAX

pytestmark = pytest.mark.gpu


def _rows_of(arrs, sample):
    pkg = product()
    sel = np.flatnonzero(np.isin(arrs["key"], sample))
    out = []
    for i in sel:
        has = bool(arrs["has_value"][i])
        vals = [int(c[i]) for c in arrs["values"]] if has else []
        out.append((int(arrs["key"][i]), pkg.AggregateWindow(int(arrs["start"][i]), int(arrs["end"][i]),
                                                             int(arrs["measure"][i]), has, vals)))
    return out


@pytest.mark.parametrize("nkeys,B,size", [(1 << 17, 1 << 21, 20), (1 << 17, 1 << 20, 7)])
def test_keyed_ooo_count_windows_at_scale_match_sampled_oracles(nkeys, B, size):
    pkg = product()
    cfg = dict(windows=[Tumbling(Count, size), Sliding(Time, 3001, 1000)], aggs=[SUM, COUNT, MIN, MAX], lateness=1000)
    op = pkg.KeyedSlicingWindowOperator(device=0)
    for a in cfg["aggs"]:
        op.addWindowFunction(a)
    op.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        op.addWindowAssigner(w)
    rng = np.random.default_rng(2025 + size)
    sample = np.sort(rng.choice(nkeys, 1200, replace=False)).astype(np.uint32)
    ora = KeyedOracle(cfg)
    total = checked = count_rows = 0
    for step in range(8):
        t_begin = 1000 + step * 1000
        keys = rng.integers(0, nkeys, B).astype(np.uint32)
        ts = t_begin + np.arange(B, dtype=np.int64) * 1000 // B
        late = rng.random(B) < 0.2
        ts = np.where(late, ts - rng.integers(1, 501, B), ts)
        vals = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
        wm = t_begin + 999 - 500
        op.processElements(keys, ts, vals)
        m = np.isin(keys, sample)
        ora.processElements(keys[m], ts[m], vals[m])
        arrs = op.processWatermarkArrays(wm)
        n = len(arrs["start"])
        total += n
        assert np.all(arrs["start"] < arrs["end"])
        if n:
            k = arrs["key"]
            assert np.count_nonzero(k[1:] != k[:-1]) + 1 == len(np.unique(k))  # a key's rows are contiguous
        count_rows += int(np.count_nonzero(arrs["measure"] == 1))
        checked += same_keyed_windows(_rows_of(arrs, sample), ora.processWatermark(wm))
        assert op.droppedCount() >= 0
    assert op.keyCount() == nkeys
    assert checked > 1200 and count_rows > nkeys
    print("rows %d (count-measure %d), sampled rows checked %d" % (total, count_rows, checked))
