"""The reference's 34 operator-level JUnit tests, transcribed 1:1.

Source: slicing/src/test/java/de/tub/dima/scotty/slicing/aggregationstore/test/windowTest/
  TumblingWindowOperatorTest.java (10), SlidingWindowOperatorTest.java (6),
  SessionWindowOperatorTest.java (10), FixedBandWindowTest.java (8).

Each case takes ``make`` (a zero-arg factory returning a fresh operator with the
reference API: addWindowFunction, addWindowAssigner, processElement,
processWatermark) so the SAME golden values pin both the CPU oracle and the
MI355X product path.  Values/positions are the reference's assertions verbatim.
"""
from specs import Tumbling, Sliding, Session, FixedBand, Time, Count, SUM, SUB


def _v(w):
    return w.getAggValues()[0]


def assert_window(w, start, end, value):  # WindowAssert.assertEquals (WindowAssert.java:10-14)
    assert w.getStart() == start and w.getEnd() == end and _v(w) == value, (w, start, end, value)


def assert_contains(ws, start, end, value):  # WindowAssert.assertContains (:16-24)
    assert any(w.getStart() == start and w.getEnd() == end and _v(w) == value for w in ws), (ws, start, end, value)


def _feed(op, pairs):
    for v, ts in pairs:
        op.processElement(v, ts)


# ------------------------------------------------------------------ TumblingWindowOperatorTest
def tumbling_inOrderTest(make):  # :25-44
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 10))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 1 and _v(r[1]) == 2
    r = op.processWatermark(55)
    assert _v(r[0]) == 3 and _v(r[1]) == 4 and _v(r[2]) == 5


def tumbling_inOrderTest2(make):  # :48-67
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 10))
    _feed(op, [(1, 0), (2, 0), (3, 20), (4, 30), (5, 40)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 3 and not r[1].hasValue()
    r = op.processWatermark(55)
    assert _v(r[0]) == 3 and _v(r[1]) == 4 and _v(r[2]) == 5


def tumbling_inOrderTwoWindowsTest(make):  # :70-93
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(Tumbling(Time, 10)); op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert [_v(r[i]) for i in range(3)] == [1, 2, 3]
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(4)] == [3, 4, 5, 7]


def tumbling_inOrderTwoWindowsDynamicTest(make):  # :95-119
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 10))
    _feed(op, [(1, 1), (2, 19)])
    op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert [_v(r[i]) for i in range(3)] == [1, 2, 3]
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(4)] == [3, 4, 5, 7]


def tumbling_inOrderTwoWindowsDynamicTest2(make):  # :121-145
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(1, 1), (2, 19)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 3
    op.addWindowAssigner(Tumbling(Time, 10))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(55)
    assert _v(r[1]) == 3 and _v(r[2]) == 4 and _v(r[3]) == 5 and _v(r[0]) == 7


def tumbling_outOfOrderTest(make):  # :148-170
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 10))
    _feed(op, [(1, 1), (1, 30), (1, 20), (1, 23), (1, 25), (1, 45)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 1 and not r[1].hasValue()
    r = op.processWatermark(55)
    assert _v(r[0]) == 3 and _v(r[1]) == 1 and _v(r[2]) == 1


def tumbling_inOrderTestCount(make):  # :174-189
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Count, 3))
    _feed(op, [(1, 1), (1, 19), (1, 29), (2, 39), (2, 49), (2, 50), (1, 51)])
    r = op.processWatermark(55)
    assert _v(r[0]) == 3 and _v(r[1]) == 6


def tumbling_outOfOrderOrderTestCount(make):  # :191-207
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Count, 3))
    _feed(op, [(1, 1), (1, 19), (1, 29), (2, 39), (2, 10), (2, 50), (1, 51)])
    r = op.processWatermark(55)
    assert _v(r[0]) == 4 and _v(r[1]) == 5


def tumbling_outOfOrderOrderTestCount2(make):  # :209-231
    op = make(); op.addWindowFunction(SUM); op.addWindowFunction(SUB)
    op.addWindowAssigner(Tumbling(Count, 3)); op.addWindowAssigner(Tumbling(Count, 5))
    _feed(op, [(1, 1), (1, 19), (1, 29), (2, 39), (1, 41), (2, 10), (2, 50), (1, 51), (3, 52)])
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(4)] == [4, 4, 6, 7]


def tumbling_outOfOrderOrderTestCount3(make):  # :233-254
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(Tumbling(Count, 3)); op.addWindowAssigner(Tumbling(Count, 5))
    _feed(op, [(1, 1), (1, 19), (1, 29), (2, 39), (1, 41), (2, 10)])
    r = op.processWatermark(30)
    assert _v(r[0]) == 4
    _feed(op, [(2, 50), (1, 51), (3, 52)])
    op.processWatermark(55)


# ------------------------------------------------------------------ SlidingWindowOperatorTest
def sliding_inOrderTest(make):  # :24-48
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Sliding(Time, 10, 5))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert _v(r[2]) == 1 and not r[1].hasValue() and _v(r[0]) == 2
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(7)] == [5, 5, 4, 4, 3, 3, 2]


def sliding_inOrderTest2(make):  # :50-74
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Sliding(Time, 10, 5))
    _feed(op, [(1, 0), (2, 0), (3, 20), (4, 30), (5, 40)])
    r = op.processWatermark(22)
    assert not r[0].hasValue() and not r[1].hasValue() and _v(r[2]) == 3
    r = op.processWatermark(55)
    assert not r[0].hasValue()
    assert [_v(r[i]) for i in range(1, 7)] == [5, 5, 4, 4, 3, 3]


def sliding_inOrderTwoWindowsTest(make):  # :77-105
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(Sliding(Time, 10, 5)); op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 2 and not r[1].hasValue() and _v(r[2]) == 1 and _v(r[3]) == 3
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(8)] == [5, 5, 4, 4, 3, 3, 2, 7]


def sliding_inOrderTwoWindowsDynamicTest(make):  # :107-136
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Sliding(Time, 10, 5))
    _feed(op, [(1, 1), (2, 19)])
    op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 2 and not r[1].hasValue() and _v(r[2]) == 1 and _v(r[3]) == 3
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(8)] == [5, 5, 4, 4, 3, 3, 2, 7]


def sliding_inOrderTwoWindowsDynamicTest2(make):  # :138-167
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Tumbling(Time, 20))
    _feed(op, [(1, 1), (2, 19)])
    r = op.processWatermark(22)
    assert _v(r[0]) == 3
    op.addWindowAssigner(Sliding(Time, 10, 5))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    r = op.processWatermark(55)
    assert [_v(r[i]) for i in range(7)] == [7, 5, 5, 4, 4, 3, 3]


def sliding_outOfOrderTest(make):  # :170-197
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Sliding(Time, 10, 5))
    _feed(op, [(1, 1), (1, 30), (1, 20), (1, 23), (1, 25), (1, 45)])
    r = op.processWatermark(22)
    assert not r[0].hasValue() and not r[1].hasValue() and _v(r[2]) == 1
    r = op.processWatermark(55)
    assert _v(r[0]) == 1 and _v(r[1]) == 1 and not r[2].hasValue()
    assert _v(r[3]) == 1 and _v(r[4]) == 2 and _v(r[5]) == 3 and _v(r[6]) == 2


# ------------------------------------------------------------------ SessionWindowOperatorTest
def session_inOrderTest(make):  # :23-43
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 1), (2, 19), (3, 23), (4, 31), (5, 49)])
    assert _v(op.processWatermark(22)[0]) == 1
    assert _v(op.processWatermark(55)[0]) == 9
    assert _v(op.processWatermark(80)[0]) == 5


def session_inOrderTestClean(make):  # :46-66
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10000))
    _feed(op, [(1, 1000), (2, 19000), (3, 23000), (4, 31000), (5, 49000)])
    assert _v(op.processWatermark(22000)[0]) == 1
    assert _v(op.processWatermark(55000)[0]) == 9
    assert _v(op.processWatermark(80000)[0]) == 5


def session_inOrderTest2(make):  # :69-87
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 0), (2, 0), (3, 20), (4, 31), (5, 42)])
    assert _v(op.processWatermark(22)[0]) == 3
    r = op.processWatermark(55)
    assert _v(r[0]) == 3 and _v(r[1]) == 4 and _v(r[2]) == 5


def session_outOfOrderTestSimpleInsert(make):  # :91-105
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 1), (1, 9), (1, 15), (1, 30), (1, 12)])
    r = op.processWatermark(50)
    assert_window(r[0], 1, 25, 4); assert_window(r[1], 30, 40, 1)


def session_outOfOrderTestRightInsert(make):  # :107-122
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 1), (1, 9), (1, 10), (1, 30), (1, 12)])
    r = op.processWatermark(50)
    assert_window(r[0], 1, 22, 4); assert_window(r[1], 30, 40, 1)


def session_outOfOrderTestLeftInsert(make):  # :124-141
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 1), (1, 9), (1, 10), (1, 30), (1, 27)])
    assert_window(op.processWatermark(22)[0], 1, 20, 3)
    assert_window(op.processWatermark(50)[0], 27, 40, 2)


def session_outOfOrderTestSplitSlice(make):  # :144-161
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 1), (1, 30), (1, 12)])
    assert_window(op.processWatermark(22)[0], 1, 11, 1)
    r = op.processWatermark(50)
    assert_window(r[0], 12, 22, 1); assert_window(r[1], 30, 40, 1)


def session_outOfOrderTestMergeSlice(make):  # :164-180
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(Session(Time, 10))
    _feed(op, [(1, 7), (1, 30), (1, 51), (1, 15), (1, 21)])
    r = op.processWatermark(70)
    assert_window(r[0], 7, 40, 4); assert_window(r[1], 51, 61, 1)


def session_outOfOrderCombinedSessionTumblingMegeSession(make):  # :182-202
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(Session(Time, 10)); op.addWindowAssigner(Tumbling(Time, 40))
    _feed(op, [(1, 7), (1, 22), (1, 51), (1, 15), (1, 37)])
    r = op.processWatermark(70)
    assert_window(r[0], 0, 40, 4); assert_window(r[1], 7, 32, 3)
    assert_window(r[2], 37, 47, 1); assert_window(r[3], 51, 61, 1)


def session_outOfOrderCombinedSessionMultiSession(make):  # :206-236
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(Session(Time, 10)); op.addWindowAssigner(Session(Time, 5))
    _feed(op, [(1, 20), (1, 40), (1, 50), (1, 57), (1, 33), (1, 31)])
    r = op.processWatermark(70)
    for s, e, v in [(20, 25, 1), (31, 38, 2), (40, 45, 1), (50, 55, 1), (57, 62, 1), (20, 30, 1), (31, 67, 5)]:
        assert_contains(r, s, e, v)


# ------------------------------------------------------------------ FixedBandWindowTest
def fixedband_inOrderTest(make):  # :27-39
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 1, 10))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    assert_window(op.processWatermark(55)[0], 1, 11, 1)


def fixedband_inOrderTest2(make):  # :41-56
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 0, 10))
    _feed(op, [(1, 0), (2, 0), (3, 20), (4, 30), (5, 40)])
    assert_window(op.processWatermark(22)[0], 0, 10, 3)
    assert op.processWatermark(55) == []


def fixedband_inOrderTest3(make):  # :58-73
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 18, 10))
    _feed(op, [(1, 0), (2, 0), (3, 20), (4, 30), (5, 40)])
    assert op.processWatermark(22) == []
    assert_window(op.processWatermark(55)[0], 18, 28, 3)


def fixedband_inOrderTwoWindowsTest(make):  # :76-94
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(FixedBand(Time, 10, 10)); op.addWindowAssigner(FixedBand(Time, 20, 10))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    assert _v(op.processWatermark(22)[0]) == 2
    assert _v(op.processWatermark(55)[0]) == 3


def fixedband_inOrderTwoWindowsTest2(make):  # :96-114
    op = make(); op.addWindowFunction(SUM)
    op.addWindowAssigner(FixedBand(Time, 14, 11)); op.addWindowAssigner(FixedBand(Time, 23, 10))
    _feed(op, [(1, 1), (2, 19), (3, 29), (4, 39), (5, 49)])
    assert _v(op.processWatermark(26)[0]) == 2
    assert _v(op.processWatermark(55)[0]) == 3


def fixedband_inOrderTwoWindowsDynamicTest(make):  # :116-135
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 10, 10))
    _feed(op, [(1, 1), (2, 19)])
    op.addWindowAssigner(FixedBand(Time, 20, 10))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    assert _v(op.processWatermark(22)[0]) == 2
    assert _v(op.processWatermark(55)[0]) == 3


def fixedband_inOrderTwoWindowsDynamicTest2(make):  # :137-155
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 10, 10))
    _feed(op, [(1, 1), (2, 19)])
    assert _v(op.processWatermark(22)[0]) == 2
    op.addWindowAssigner(FixedBand(Time, 20, 21))
    _feed(op, [(3, 29), (4, 39), (5, 49)])
    assert _v(op.processWatermark(55)[0]) == 7


def fixedband_outOfOrderTest(make):  # :158-177
    op = make(); op.addWindowFunction(SUM); op.addWindowAssigner(FixedBand(Time, 10, 20))
    _feed(op, [(1, 1), (1, 29), (1, 20), (1, 23), (1, 25), (1, 45)])
    assert op.processWatermark(22) == []
    assert _v(op.processWatermark(55)[0]) == 4


TUMBLING_TIME = [tumbling_inOrderTest, tumbling_inOrderTest2, tumbling_inOrderTwoWindowsTest,
                 tumbling_inOrderTwoWindowsDynamicTest, tumbling_inOrderTwoWindowsDynamicTest2,
                 tumbling_outOfOrderTest]
TUMBLING_COUNT = [tumbling_inOrderTestCount, tumbling_outOfOrderOrderTestCount,
                  tumbling_outOfOrderOrderTestCount2, tumbling_outOfOrderOrderTestCount3]
SLIDING = [sliding_inOrderTest, sliding_inOrderTest2, sliding_inOrderTwoWindowsTest,
           sliding_inOrderTwoWindowsDynamicTest, sliding_inOrderTwoWindowsDynamicTest2, sliding_outOfOrderTest]
SESSION = [session_inOrderTest, session_inOrderTestClean, session_inOrderTest2, session_outOfOrderTestSimpleInsert,
           session_outOfOrderTestRightInsert, session_outOfOrderTestLeftInsert, session_outOfOrderTestSplitSlice,
           session_outOfOrderTestMergeSlice, session_outOfOrderCombinedSessionTumblingMegeSession,
           session_outOfOrderCombinedSessionMultiSession]
FIXED_BAND = [fixedband_inOrderTest, fixedband_inOrderTest2, fixedband_inOrderTest3, fixedband_inOrderTwoWindowsTest,
              fixedband_inOrderTwoWindowsTest2, fixedband_inOrderTwoWindowsDynamicTest,
              fixedband_inOrderTwoWindowsDynamicTest2, fixedband_outOfOrderTest]
ALL = TUMBLING_TIME + TUMBLING_COUNT + SLIDING + SESSION + FIXED_BAND
assert len(ALL) == 34
