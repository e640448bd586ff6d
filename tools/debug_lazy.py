"""Locate the first divergence of a LazySlice-records operator (tests/test_gpu_exact.py configs) from the oracle:
replays the stream one tuple-push at a time and compares the slice lists (tStart, tEnd, tLast, cStart, cLast,
records) after every tuple.  GPU debugging aid."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import product, build_ops  # noqa: E402
from specs import *  # noqa: E402,F401,F403

pkg = product()


def _nz(x):
    return x + 1 if x & (x - 1) == 0 else x


def gpu_slices(op):
    f = op._l.scotty_debug_dump
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    op.sync()
    buf = np.zeros(1 << 22, dtype=np.int64)
    n = f(op._h, 0, buf.ctypes.data, len(buf))
    v = buf[:n].tolist()
    S = v[0]
    cols = [v[1 + k * S: 1 + (k + 1) * S] for k in range(7)]  # ts te tl cnt cs cl ty
    p = 1 + 7 * S
    nctx = v[p]; p += 1
    for _ in range(nctx):
        ns = v[p]; p += 1 + 2 * ns
    meta = v[p:p + 10]
    p += 10
    gpu_slices.meta = meta
    rlo, rhi, nn = v[p:p + S], v[p + S:p + 2 * S], v[p + 2 * S:p + 3 * S]
    p += 3 * S
    rend = v[p]; p += 1
    recs = v[p:p + 2 * rend]
    rts = recs[0::2]
    out = []
    for i in range(S):
        out.append((cols[0][i], cols[1][i], cols[2][i], cols[4][i], cols[5][i], cols[3][i], nn[i],
                    tuple(rts[rlo[i]:rhi[i]])))
    return out


def ora_slices(ora):
    out = []
    for i in range(ora.store_size()):
        s = ora.slice(i)
        vals = ora.slice_values(i)
        out.append((s.t_start, s.t_end, s.t_last, s.c_start, s.c_last, None, 1 if vals else 0,
                    tuple(ora.slice_records(i))))
    return out


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    rng = np.random.default_rng(9700 + seed)
    vt = ["i32", "i32", "i64", "f64"][seed % 4]
    wins = [Tumbling(Count, int(rng.integers(1, 40)))]
    if rng.random() < 0.5:
        size = int(rng.integers(2, 60))
        wins.append(Sliding(Count, size, int(rng.integers(1, size + 1))))
    if rng.random() < 0.4:
        wins.append(Tumbling(Time, _nz(int(rng.integers(5, 100)))))
    if rng.random() < 0.25:
        wins.append(Session(Time, int(rng.integers(5, 100))))
    rng.shuffle(wins)
    import test_gpu_exact as T
    aggs = T._lazy_aggs(rng, vt, invertible=seed % 3 == 2)
    cfg = dict(windows=wins, aggs=aggs, lateness=int(rng.choice([10, 100, 1000])))
    n = int(rng.integers(200, 6000))
    ts, vals = pkg.workloads.stream(n, [0.5, 1, 3, 8][seed % 4], t0=int(rng.integers(0, 500)),
                                    ooo_frac=[0.02, 0.1, 0.3][seed % 3], max_delay=int(rng.integers(1, 60)),
                                    seed=seed, value_type=vt, gaps=T._gaps(rng, n, 400, 10, 150))
    print("cfg", cfg, "n", n)
    from helpers import interval_schedule, same_windows
    sched = interval_schedule(ts, int(rng.integers(1, 6)), lag=int(rng.integers(0, 60)),
                              pushes_per_interval=int(rng.integers(1, 3)))
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    gpu, ora = build_ops(cfg, vt)
    for st in sched:
        if st[0] == "push":
            lo, hi = st[1], st[2]
            step = chunk or (hi - lo)
            for a in range(lo, hi, step):
                b = min(hi, a + step)
                gpu.processElements(ts[a:b], vals[a:b])
                ora.processElements(ts[a:b], vals[a:b])
                g = [x[:5] + x[6:] for x in gpu_slices(gpu)]
                o = [x[:5] + x[6:] for x in ora_slices(ora)]
                if g != o:
                    print("DIVERGED after push [%d,%d)" % (a, b), "ts", ts[a:b][:80].tolist())
                    shown = 0
                    for k in range(max(len(g), len(o))):
                        x = g[k] if k < len(g) else None
                        y = o[k] if k < len(o) else None
                        if x != y and shown < 6:
                            print("  slice", k, "\n   gpu", x, "\n   ora", y)
                            shown += 1
                    return
        else:
            before = gpu_slices(gpu)
            wa = gpu.processWatermark(st[1])
            wb = ora.processWatermark(st[1])
            try:
                same_windows(wa, wb)
            except AssertionError as e:
                print("WINDOWS DIVERGED at wm", st[1], str(e)[:300])
                gpu_slices(gpu)
                print("meta after wm (maxEventTime nextEdgeTs currentCount unsorted head tail wlo whi lastWm lastCount)",
                      gpu_slices.meta)
                for k, x in enumerate(before):
                    if x[0] >= 1100 and x[0] <= 1200:
                        print("  slice", k, x[:7], "nrec", len(x[7]), x[7][:8])
                return
    print("no divergence")


if __name__ == "__main__":
    main()
