"""The oracle's first-partial aggregation (ORC_AGG_FIRST): the arrival index of the tuple whose fields a combine that
keeps partialAggregate1 leaves in the window's result (B/flinkBenchmark/aggregations/SumAggregation.java:16-18,
D/flink-demo/.../SumWindowFunction.java:16-17).  AggregateValueState lifts a slice's first element and folds later ones
into it (S/state/AggregateValueState.java:23-31); a window's state clones the first non-empty slice's partial and folds
the rest into it, in slice order (:55-69) -- so the window's value is the first tuple added to its first non-empty
slice, which for out-of-order input is not the window's earliest-arriving tuple.  Hand-computed cases (CPU)."""
import numpy as np

from helpers import ROOT  # noqa: F401  (sys.path)
from oracle.oracle import OracleOperator, AGG_FIRST
from specs import Tumbling, Time, SUM


def _op(windows, aggs, lateness=100):
    o = OracleOperator()
    for a in aggs:
        o.addWindowFunction(a)
    o.setMaxLateness(lateness)
    for w in windows:
        o.addWindowAssigner(w)
    return o


def _rows(ws):
    return [(w.getStart(), w.getEnd(), w.getAggValues()) for w in ws]


def test_first_in_order_is_the_windows_first_tuple():
    o = _op([Tumbling(Time, 10)], [SUM, AGG_FIRST])
    o.processElements(np.array([1, 2, 12, 15], np.int64), np.array([5, 6, 7, 8], np.int64))
    assert _rows(o.processWatermark(22)) == [(0, 10, [11, 0]), (10, 20, [15, 2])]


def test_first_out_of_order_is_the_first_non_empty_slices_first_tuple():
    # Tumbling 10 + 5: slices [0,5) [5,10).  Tuple 0 (ts 6) opens [5,10); tuple 1 (ts 2) is late and lands in [0,5).
    # Window [0,10): its first non-empty slice in slice order is [0,5), whose first tuple is #1 -- not #0, the
    # window's earliest arrival.
    o = _op([Tumbling(Time, 10), Tumbling(Time, 5)], [SUM, AGG_FIRST])
    o.processElements(np.array([0, 6, 2], np.int64), np.array([0, 10, 20], np.int64))
    rows = {(s, e): v for s, e, v in _rows(o.processWatermark(11))}
    assert rows[(0, 10)] == [30, 0]   # slices [0,5) {ts 0 (#0), ts 2 (#2)} and [5,10) {#1}: the first slice's first: #0
    o2 = _op([Tumbling(Time, 10), Tumbling(Time, 5)], [SUM, AGG_FIRST])
    o2.processElements(np.array([6, 2], np.int64), np.array([10, 20], np.int64))
    rows2 = {(s, e): v for s, e, v in _rows(o2.processWatermark(11))}
    assert rows2[(0, 10)] == [30, 1]  # [0,5) holds only #1 (late) and precedes [5,10): #1, not the earlier #0
    assert rows2[(0, 5)] == [20, 1] and rows2[(5, 10)] == [10, 0]


def test_first_counts_dropped_tuples_in_the_arrival_index():
    # a too-late tuple throws in the reference after WindowManager.incrementCount: it still takes an arrival index
    o = _op([Tumbling(Time, 10)], [AGG_FIRST], lateness=1)
    o.processElements(np.array([100, 101], np.int64), np.array([1, 1], np.int64))
    o.processWatermark(105)
    assert o.processElements(np.array([3, 112], np.int64), np.array([1, 1], np.int64)) == 1  # #2 dropped
    rows = _rows(o.processWatermark(130))
    assert (110, 120, [3]) in rows
