"""Pins the CPU oracle to the reference's own 48 JUnit tests (CPU only).

Operator-level (34): tests/junit_cases.py.  Component-level (14), transcribed here:
  T/SliceManagerTest.java (6), T/SliceFactoryTest.java (4), T/LazyAggregateStoreTest.java (4)
with T = slicing/src/test/java/de/tub/dima/scotty/slicing/aggregationstore/test/.
"""
import pytest

import junit_cases
from oracle.oracle import (OracleOperator, STATE_MOCK, WIN_TEST_SCRIPTED, WIN_TEST_NULLCTX, WIN_SESSION, TIME,
                           COUNT as M_COUNT, AGG_SUM_I32, JavaError)


@pytest.mark.parametrize("case", junit_cases.ALL, ids=lambda c: c.__name__)
def test_operator_junit(case):
    case(OracleOperator)


@pytest.mark.parametrize("case", junit_cases.ALL, ids=lambda c: c.__name__)
@pytest.mark.parametrize("order", [1, 2])
def test_operator_junit_mod_order_neutral(case, order):
    """Set<WindowModifications> is an identity-hashed HashSet (S/SliceManager.java:90): its
    iteration order is unspecified.  The golden values must hold under any order."""
    def make():
        op = OracleOperator()
        op.setModOrder(order, seed=7)
        return op
    case(make)


# ------------------------------------------------------------------ SliceManagerTest (StateFactoryMock)
def _sm():
    op = OracleOperator(STATE_MOCK)
    op.addWindowFunction(AGG_SUM_I32)               # :45-50
    op.addWindowAssigner(WIN_TEST_SCRIPTED, TIME, 0, 0)
    return op


def check_records(values, records):
    """SliceManagerTest.checkRecords (:289-295): every record must equal values[i++] in order; the
    trailing assertFalse(hasNext()) is vacuous, so the records form a PREFIX of ``values``
    (AddModificationSplitTest lists a ts 30 that was never inserted)."""
    assert len(records) <= len(values) and list(records) == list(values[:len(records)]), (records, values)


def _chk(op, i, start, end, first, last):
    s = op.slice(i)
    assert (s.t_start, s.t_end, s.t_first, s.t_last) == (start, end, first, last), (i, s.t_start, s.t_end,
                                                                                      s.t_first, s.t_last)


def test_ShiftLowerModificationTest():  # :56-89
    op = _sm()
    op.store_append_new_slice(0, 10)
    for ts in (1, 4, 8, 9):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(10, 20)
    for ts in (14, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30)
    op.manager_process_element(1, 24)
    op.manager_process_element(1, 5)
    _chk(op, 0, 0, 5, 1, 4)
    _chk(op, 1, 5, 20, 5, 19)
    check_records([5, 8, 9, 14, 19], op.slice_records(1))


def test_ShiftHigherModificationTest():  # :94-125
    op = _sm()
    op.store_append_new_slice(0, 10)
    op.manager_process_element(1, 1)
    op.store_append_new_slice(10, 20)
    for ts in (12, 14, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30)
    op.manager_process_element(1, 24)
    op.manager_process_element(1, 15)
    _chk(op, 0, 0, 15, 1, 14)
    _chk(op, 1, 15, 20, 15, 19)
    check_records([1, 12, 14, 15], op.slice_records(0))


def test_ShiftModificationSplitTest():  # :130-170
    op = _sm()
    op.store_append_new_slice(0, 10, fixed=False, flex_count=2)
    assert op.slice(0).flex_count == 2 and not op.slice(0).type_fixed  # not movable
    for ts in (1, 4, 8, 9):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(10, 20, flex_count=2)
    for ts in (14, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30, flex_count=2)
    op.manager_process_element(1, 24)
    op.manager_process_element(1, 5)
    _chk(op, 0, 0, 5, 1, 4)
    _chk(op, 1, 5, 10, 5, 9)
    _chk(op, 2, 10, 20, 14, 19)
    check_records([5, 8, 9], op.slice_records(1))


def test_ShiftModificationSplitTest2():  # :175-214
    op = _sm()
    op.store_append_new_slice(0, 10, flex_count=2)
    op.manager_process_element(1, 1)
    op.store_append_new_slice(10, 20, flex_count=2)
    for ts in (12, 14, 17, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30, flex_count=2)
    op.manager_process_element(1, 24)
    op.manager_process_element(1, 15)
    _chk(op, 0, 0, 10, 1, 1)
    _chk(op, 1, 10, 15, 12, 14)
    _chk(op, 2, 15, 20, 15, 19)
    check_records([15, 17, 19], op.slice_records(2))


def test_AddModificationSplitTest():  # :219-251
    op = _sm()
    op.store_append_new_slice(0, 10)
    op.manager_process_element(1, 1)
    op.store_append_new_slice(10, 20)
    for ts in (14, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30)
    for ts in (22, 24, 26, 27):
        op.manager_process_element(1, ts)
    op.manager_process_element(1, 25)
    _chk(op, 2, 20, 25, 22, 24)
    _chk(op, 3, 25, 30, 25, 27)
    check_records([25, 26, 27, 30], op.slice_records(3))


def test_DeleteModificationTest():  # :256-287
    op = _sm()
    op.store_append_new_slice(0, 10)
    op.manager_process_element(1, 1)
    op.store_append_new_slice(10, 20)
    for ts in (14, 19):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(20, 30)
    op.manager_process_element(1, 24)
    op.store_append_new_slice(30, 35)
    for ts in (31, 33):
        op.manager_process_element(1, ts)
    op.store_append_new_slice(35, 45)
    op.manager_process_element(1, 38)
    op.manager_process_element(1, 35)
    _chk(op, 2, 20, 35, 24, 33)
    _chk(op, 3, 35, 45, 35, 38)
    check_records([24, 31, 33], op.slice_records(2))


# ------------------------------------------------------------------ SliceFactoryTest
def _sf():
    op = OracleOperator(STATE_MOCK)
    op.addWindowFunction(AGG_SUM_I32)
    return op


def test_LazySliceTest():  # :422-433
    op = _sf()
    op.addWindowAssigner(WIN_TEST_NULLCTX, TIME, 0, 0)
    f = op.flags()
    assert op.max_lateness() > 0 and f["hasContextAwareWindow"] and not f["isSessionWindowCase"]
    assert op.factory_would_be_lazy()


def test_LazySliceTestCount():  # :439-448
    op = _sf()
    op.addWindowAssigner(WIN_TEST_NULLCTX, M_COUNT, 0, 0)
    assert op.flags()["hasCountMeasure"]
    assert op.factory_would_be_lazy()


def test_EagerSliceTestSession():  # :453-472
    op = _sf()
    op.addWindowAssigner(WIN_SESSION, TIME, 1000, 0)
    f = op.flags()
    assert op.max_lateness() > 0 and f["hasContextAwareWindow"] and f["isSessionWindowCase"]
    assert not f["hasCountMeasure"]
    assert not op.factory_would_be_lazy()
    op.addWindowAssigner(WIN_SESSION, TIME, 2000, 0)
    assert op.flags()["isSessionWindowCase"]
    assert not op.factory_would_be_lazy()


def test_LazySliceTestContextAware():  # :478-490
    op = _sf()
    op.addWindowAssigner(WIN_SESSION, TIME, 1000, 0)
    op.addWindowAssigner(WIN_TEST_NULLCTX, TIME, 0, 0)
    f = op.flags()
    assert op.max_lateness() > 0 and f["hasContextAwareWindow"] and not f["isSessionWindowCase"]
    assert op.factory_would_be_lazy()


# ------------------------------------------------------------------ LazyAggregateStoreTest (StateFactoryMock)
def _ls(ends):
    op = OracleOperator(STATE_MOCK)
    op.addWindowFunction(AGG_SUM_I32)
    for s, e in ends:
        op.store_append_new_slice(s, e, fixed=True)
    return op


def test_getSliceByIndex():  # :38-57
    spec = [(0, 10), (10, 20), (20, 30), (40, 50)]
    op = _ls(spec)
    for i, (s, e) in enumerate(spec):
        assert (op.slice(i).t_start, op.slice(i).t_end) == (s, e)
    assert op.store_size() == 4 and op.slice(3).t_start == 40  # getCurrentSlice()


def test_findSliceByTs():  # :59-78
    spec = [(0, 10), (10, 20), (20, 30), (40, 50)]
    op = _ls(spec)
    for i, (s, e) in enumerate(spec):
        assert op.find_slice_index_by_ts(s) == i
        assert op.find_slice_index_by_ts(e - 1) == i
        assert op.find_slice_index_by_ts(s + 5) == i


def test_insertValue():  # :81-99
    op = _ls([(0, 10), (10, 20), (20, 30), (40, 50)])
    op.insert_value_to_slice(1, 1, 14)
    op.insert_value_to_slice(2, 2, 22)
    op.insert_value_to_current(3, 22)
    assert op.slice_values(0)[0] is None        # mock ValueState: never empty, value null
    assert op.slice_values(1)[0] == 1


def test_aggregateWindow():  # :101-121 (the reference asserts nothing after building the windows)
    op = _ls([(0, 10), (10, 20), (20, 30), (30, 40)])
    op.insert_value_to_slice(1, 1, 14)
    op.insert_value_to_slice(2, 2, 22)
    op.insert_value_to_current(3, 33)
    assert op.store_size() == 4


def test_error_semantics_too_late_tuple():
    """A tuple older than the oldest slice: findSliceIndexByTimestamp -> -1 and ArrayList.get(-1)
    throws (S/aggregationstore/LazyAggregateStore.java:29-37, S/SliceManager.java:75-76)."""
    op = OracleOperator()
    op.addWindowFunction(AGG_SUM_I32)
    op.addWindowAssigner(0, TIME, 10, 0)
    op.processElement(1, 5)
    with pytest.raises(JavaError) as ei:
        op.processElement(1, -3)
    assert ei.value.code == -1


def test_error_semantics_empty_session_context():
    """SessionContext.triggerWindows calls getWindow(0) on an empty context (C/windowType/SessionWindow.java:108)."""
    op = OracleOperator()
    op.addWindowFunction(AGG_SUM_I32)
    op.addWindowAssigner(WIN_SESSION, TIME, 10, 0)
    op.processElement(1, 1)
    op.processWatermark(100)          # triggers [1,11) and empties the context
    with pytest.raises(JavaError):
        op.processWatermark(200)
