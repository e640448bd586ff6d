"""Key-hash router of the keyed operator over G ranks (scotty_route_keyed) -- host-only product
code, so it runs here without a GPU.  Checked against a plain-Python restatement of the SPE's key-group assignment
(Flink KeyGroupRangeAssignment: murmurHash(key.hashCode()) % maxParallelism, then keyGroup * G / maxParallelism; the
routing in front of F/KeyedScottyWindowOperator.java:56-66).  No JVM is available to run the SPE itself, so the
murmur restatement is "parity unpinned" against Flink; what is pinned is the split's contract: a partition of the
batch, stable per shard, and a pure function of the key."""
import numpy as np
import pytest

from helpers import product


def murmur_java(code):
    """MathUtils.murmurHash(int) with Java int wrap (test-side restatement)."""
    M = 0xFFFFFFFF
    c = code & M
    c = (c * 0xCC9E2D51) & M
    c = ((c << 15) | (c >> 17)) & M
    c = (c * 0x1B873593) & M
    c = ((c << 13) | (c >> 19)) & M
    c = (c * 5 + 0xE6546B64) & M
    c ^= 4
    c ^= c >> 16
    c = (c * 0x85EBCA6B) & M
    c ^= c >> 13
    c = (c * 0xC2B2AE35) & M
    c ^= c >> 16
    s = c - (1 << 32) if c >= 1 << 31 else c
    if s >= 0:
        return s
    return -s if s != -(1 << 31) else 0


def shard_py(key, world, maxp=128):
    return (murmur_java(key) % maxp) * world // maxp


@pytest.fixture(scope="module")
def pkg():
    return product()


def test_key_shard_matches_restatement(pkg):
    rng = np.random.default_rng(3)
    keys = [0, 1, 2, 42, 2**31 - 1, 2**31, 2**32 - 1] + [int(x) for x in rng.integers(0, 2**32, 2000)]
    for world, maxp in [(1, 128), (2, 128), (3, 128), (8, 128), (8, 4096), (128, 128), (5, 7)]:
        r = pkg.KeyedShardRouter(world, maxp)
        for k in keys:
            assert r.shardOf(k) == shard_py(k, world, maxp), (k, world, maxp)


def test_key_shard_rejects_bad_world(pkg):
    L = pkg.lib()
    assert L.scotty_key_shard(5, 0, 128) < 0
    assert L.scotty_key_shard(5, 200, 128) < 0
    with pytest.raises(ValueError):
        pkg.KeyedShardRouter(129, 128)


@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float64])
@pytest.mark.parametrize("world", [1, 2, 8])
def test_route_is_stable_partition(pkg, dtype, world):
    rng = np.random.default_rng(world)
    n = 50_000
    keys = rng.integers(0, 1_000_000, size=n).astype(np.uint32)
    ts = np.arange(n, dtype=np.int64) * 3 - rng.integers(0, 500, size=n)  # out of order: arrival order matters
    vals = rng.integers(-1000, 1000, size=n).astype(dtype)
    parts = pkg.KeyedShardRouter(world).route(keys, ts, vals)
    sh = np.array([shard_py(int(k), world) for k in keys])
    assert sum(len(p[0]) for p in parts) == n
    for r, (k, t, v) in enumerate(parts):
        m = sh == r
        assert np.array_equal(k, keys[m]) and np.array_equal(t, ts[m]) and np.array_equal(v, vals[m])
        assert v.dtype == vals.dtype


def test_route_threads_agree_and_balance(pkg):
    """Multi-threaded scatter (per-thread histograms) == one thread, on a batch large enough to split; uniform keys
    spread evenly over 8 ranks (the keyed path's near-linear scaling assumes it)."""
    rng = np.random.default_rng(11)
    n = 1 << 21
    keys = rng.integers(0, 1_000_000, size=n).astype(np.uint32)
    ts = np.arange(n, dtype=np.int64)
    vals = rng.integers(-5, 5, size=n).astype(np.int32)
    a = pkg.KeyedShardRouter(8, threads=1).route(keys, ts, vals)
    b = pkg.KeyedShardRouter(8, threads=7).route(keys, ts, vals)
    for x, y in zip(a, b):
        for u, w in zip(x, y):
            assert np.array_equal(u, w)
    sizes = np.array([len(p[0]) for p in a])
    assert sizes.sum() == n and sizes.min() > 0.9 * n / 8 and sizes.max() < 1.1 * n / 8
    # every key lands on exactly one rank
    owners = {}
    for r, (k, _, _) in enumerate(a):
        for key in np.unique(k)[:2000]:
            assert owners.setdefault(int(key), r) == r


def test_route_empty_and_single(pkg):
    r = pkg.KeyedShardRouter(4)
    parts = r.route(np.zeros(0, np.uint32), np.zeros(0, np.int64), np.zeros(0, np.int32))
    assert [len(p[0]) for p in parts] == [0, 0, 0, 0]
    parts = r.route(np.array([7], np.uint32), np.array([5], np.int64), np.array([9], np.int32))
    s = shard_py(7, 4)
    assert [len(p[0]) for p in parts] == [1 if i == s else 0 for i in range(4)]
    assert parts[s][2][0] == 9
