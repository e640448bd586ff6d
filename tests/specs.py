"""Window / aggregation specs shared by the oracle and the product parity tests.

Mirrors the reference's window value types (C/windowType/TumblingWindow.java,
SlidingWindow.java, SessionWindow.java, FixedBandWindow.java) and WindowMeasure.
"""
from collections import namedtuple

Time, Count = 0, 1
WindowSpec = namedtuple("WindowSpec", "kind measure a b")


def Tumbling(measure, size):
    return WindowSpec(0, measure, size, 0)


def Sliding(measure, size, slide):
    return WindowSpec(1, measure, size, slide)


def Session(measure, gap):
    return WindowSpec(2, measure, gap, 0)


def FixedBand(measure, start, size):
    return WindowSpec(3, measure, start, size)


# aggregate kinds (oracle/scotty_oracle.h, include/scotty_mi355x.h share the numbering)
SUM, COUNT, MIN, MAX = 0, 1, 2, 3
SUM_I64, MIN_I64, MAX_I64 = 4, 5, 6
SUM_F64, MIN_F64, MAX_F64 = 7, 8, 9
SUB = 100          # (a,b)->a-b, TumblingWindowOperatorTest.java:212
INVERTIBLE = 0x10000
