"""Synthetic workloads of the reference's benchmark configurations (BASELINE.json configs).

Window definitions follow the reference generators exactly (java.util.Random restated):
  randomTumbling(n, min, max)  benchmark/src/main/java/de/tub/dima/scotty/flinkBenchmark/BenchmarkRunner.java:136-151
Tuple streams are seeded numpy streams of the same shape as LoadGeneratorSource / TimeStampGenerator
(B/flinkBenchmark/LoadGeneratorSource.java:79, D/beam-demo/.../TimeStampGenerator.java:42-46).
"""
import numpy as np

_MASK = (1 << 48) - 1
_MULT = 0x5DEECE66D


class JavaRandom:
    """java.util.Random (48-bit LCG) -- nextInt, nextInt(bound), nextDouble, nextLong."""

    def __init__(self, seed):
        self.seed = (seed ^ _MULT) & _MASK

    def next(self, bits):
        self.seed = (self.seed * _MULT + 0xB) & _MASK
        r = self.seed >> (48 - bits)
        if r & (1 << (bits - 1)) and bits == 32:
            r -= 1 << 32
        return r

    def nextInt(self, bound=None):
        if bound is None:
            return self.next(32)
        if bound & (-bound) == bound:
            return (bound * self.next(31)) >> 31
        while True:
            bits = self.next(31)
            val = bits % bound
            if bits - val + (bound - 1) < (1 << 31):
                return val

    def nextDouble(self):
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))


class JavaRandomInts:
    """java.util.Random.nextInt() as numpy int32 blocks (C1: Random(43).nextInt() values).  The
    48-bit LCG seed_{k+1} = a*seed_k + c jumps k steps as seed_k = A_k*seed_0 + C_k (mod 2^48); uint64 arithmetic
    wraps mod 2^64, which 2^48 divides, so the masked products are exact."""

    _B = 1 << 16

    def __init__(self, seed):
        self.seed = np.uint64((seed ^ _MULT) & _MASK)
        a = np.zeros(self._B, np.uint64)
        c = np.zeros(self._B, np.uint64)
        x, y = 1, 0
        for k in range(self._B):  # A_{k+1}, C_{k+1}: k+1 steps from seed_0
            x, y = (x * _MULT) & _MASK, (y * _MULT + 0xB) & _MASK
            a[k], c[k] = x, y
        self._a, self._c = a, c

    def next_ints(self, n):
        out = np.empty(n, np.int32)
        m = np.uint64(_MASK)
        with np.errstate(over="ignore"):
            for b0 in range(0, n, self._B):
                k = min(self._B, n - b0)
                seeds = (self._a[:k] * self.seed + self._c[:k]) & m
                out[b0:b0 + k] = (seeds >> np.uint64(16)).astype(np.uint32).view(np.int32)
                self.seed = seeds[k - 1]
        return out


def random_tumbling_sizes(n=1000, lo=1, hi=20, seed=10):
    """BenchmarkRunner.getAssigner("randomTumbling(n,lo,hi)"): sizes in ms, Random(10)."""
    r = JavaRandom(seed)
    out = []
    for _ in range(n):
        size = lo + r.nextDouble() * (hi - lo)
        out.append(int(size * 1000))
    return out


def random_count_sizes(n=1000, lo=1, hi=20, seed=10):
    """BenchmarkRunner.getAssigner("randomCount(n,lo,hi)"): TumblingWindow(Count, (int) size), Random(10)."""
    r = JavaRandom(seed)
    return [int(lo + r.nextDouble() * (hi - lo)) for _ in range(n)]


def stream(n, rate_per_ms, t0=0, ooo_frac=0.0, max_delay=0, seed=0, value_type="i32", gaps=None):
    """Arrival-ordered (ts, value) columns.

    Event time advances by 1 ms every ``rate_per_ms`` tuples starting at t0; a fraction ``ooo_frac`` of
    tuples is late by U[1, max_delay] ms (clamped to >= 1, as TimeStampGenerator does).  ``gaps`` is an
    optional list of (at_tuple_index, silence_ms) session silences.
    """
    rng = np.random.default_rng(seed)
    idx = np.arange(n, dtype=np.int64)
    ts = t0 + idx // int(rate_per_ms) if rate_per_ms >= 1 else t0 + (idx * int(round(1.0 / rate_per_ms)))
    if gaps:
        shift = np.zeros(n, dtype=np.int64)
        for at, ms in gaps:
            shift[at:] += ms
        ts = ts + shift
    if ooo_frac > 0 and max_delay > 0:
        late = rng.random(n) < ooo_frac
        d = rng.integers(1, max_delay + 1, size=n)
        ts = np.where(late, np.maximum(ts - d, 1), ts)
    if value_type == "i32":
        vals = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    elif value_type == "i64":
        vals = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)
    else:
        vals = rng.standard_normal(n) * 1000.0
    return ts.astype(np.int64), vals
