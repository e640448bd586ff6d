"""Bisect the smallest failing prefix of a test config (batch-parallel vs serial replay vs oracle)."""
import sys, os, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import product, build_ops, interval_schedule
from specs import *
pkg = product()

def _nz(x): return x + 1 if x & (x - 1) == 0 else x

def cfg_count(seed):
    rng = np.random.default_rng(9100 + seed)
    wins = [Tumbling(Count, int(rng.integers(1, 50)))]
    if rng.random() < 0.5:
        size = int(rng.integers(2, 60)); wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
    if rng.random() < 0.5: wins.append(Tumbling(Time, _nz(int(rng.integers(5, 100)))))
    if rng.random() < 0.3: wins.append(Session(Time, int(rng.integers(5, 100))))
    cfg = dict(windows=wins, aggs=[SUM, COUNT, MAX], lateness=int(rng.choice([1, 10, 1000])))
    n = int(rng.integers(10, 5000))
    gaps = [(int(i), int(rng.integers(10, 200))) for i in range(300, n, 300)]
    ts, vals = pkg.workloads.stream(n, [0.5, 1, 3][seed % 3], t0=int(rng.integers(0, 500)), seed=seed, gaps=gaps)
    return cfg, ts, vals, int(rng.integers(1, 6)), int(rng.integers(0, 20))

import ctypes
def dump(op):
    L = op._l
    f = L.scotty_debug_dump; f.restype = ctypes.c_int64; f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    op.sync()
    buf = np.zeros(1 << 22, dtype=np.int64)
    n = f(op._h, 0, buf.ctypes.data, len(buf))
    v = buf[:n].tolist(); S = v[0]; cols = [v[1 + k * S: 1 + (k + 1) * S] for k in range(7)]
    rest = v[1 + 7 * S:]
    slices = list(zip(*cols))
    return slices, rest

def run(cfg, ts, vals, nint, lag, serial, stop_at_wm=None):
    op = pkg.SlicingWindowOperator(device=0)
    op.tune("exact_serial", serial)
    for a in cfg["aggs"]: op.addWindowFunction(a)
    op.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]: op.addWindowAssigner(w)
    out = []
    for st in interval_schedule(ts, nint, lag=lag):
        if st[0] == "push": op.processElements(ts[st[1]:st[2]], vals[st[1]:st[2]])
        else:
            if stop_at_wm is not None and len(out) == stop_at_wm:
                print("  serial" if serial else "  batch", "dropped", op.droppedCount(), "processed", op.processedCount())
                return dump(op)
            out.append([w.key() for w in op.processWatermark(st[1])])
    return out

def cfg_bvs(seed):
    rng = np.random.default_rng(4400 + seed)
    wins = [Session(Time, int(rng.integers(3, 300)))]
    if rng.random() < 0.3: wins.append(Session(Time, int(rng.integers(3, 300))))
    for _ in range(int(rng.integers(0, 3))):
        if rng.random() < 0.5: wins.append(Tumbling(Time, _nz(int(rng.integers(5, 200)))))
        else:
            size = int(rng.integers(10, 300)); wins.append(Sliding(Time, size, _nz(int(rng.integers(3, size + 1)))))
    rng.shuffle(wins)
    aggs = [a for a in [SUM, COUNT, MIN, MAX] if rng.random() < 0.7] or [SUM]
    cfg = dict(windows=wins, aggs=aggs, lateness=int(rng.choice([1, 5, 50, 500, 1000])))
    n = 400_000
    every = int(rng.integers(5_000, 50_000))
    gaps = [(int(i), int(rng.integers(100, 3000))) for i in range(every, n, every)]
    ts, vals = pkg.workloads.stream(n, [2, 10, 40][seed % 3], t0=500, ooo_frac=[0.05, 0.2][seed % 2],
                                    max_delay=int(rng.integers(10, 600)), seed=seed, gaps=gaps)
    return cfg, ts, vals, 6, 300

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
which = sys.argv[2] if len(sys.argv) > 2 else "count"
cfg, ts, vals, nint, lag = (cfg_count if which == "count" else cfg_bvs)(seed)
print("cfg", cfg, "n", len(ts), "nint", nint, "lag", lag)
def bad(n):
    a = run(cfg, ts[:n], vals[:n], nint, lag, 0); b = run(cfg, ts[:n], vals[:n], nint, lag, 1)
    return a != b
lo, hi = 1, len(ts)
if not bad(hi): print("no failure"); sys.exit(0)
while hi - lo > 1:
    mid = (lo + hi) // 2
    if bad(mid): hi = mid
    else: lo = mid
n = hi
print("smallest failing n", n)
a = run(cfg, ts[:n], vals[:n], nint, lag, 0); b = run(cfg, ts[:n], vals[:n], nint, lag, 1)
for i, (x, y) in enumerate(zip(a, b)):
    if x != y:
        print("wm", i); print(" batch ", x[:20]); print(" serial", y[:20]); break
print("ts tail", ts[max(0, n-30):n].tolist())
for k in range(len(a)):
    if a[k] != b[k]:
        for x, y in zip(a[k], b[k]):
            if x != y: print("first diff", x, y); break
        sa, ra = run(cfg, ts[:n], vals[:n], nint, lag, 0, stop_at_wm=k)
        sb, rb = run(cfg, ts[:n], vals[:n], nint, lag, 1, stop_at_wm=k)
        print("slices batch", len(sa), "serial", len(sb))
        for i, (x, y) in enumerate(zip(sa, sb)):
            if x != y: print(" slice", i, "batch", x, "serial", y)
        print("rest batch", ra[:40]); print("rest serial", rb[:40])
        break
