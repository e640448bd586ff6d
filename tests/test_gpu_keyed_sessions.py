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
