"""Timing of the exact engine on BASELINE configs[2] (C3, non-keyed sliding+session, 20% OOO, MIN/MAX) and
configs[3] (C4, keyed sliding 60s/1s SUM over 1M keys).  Inputs resident in HBM; results stay in HBM."""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("scotty-window-processor_amd")
Tumbling, Sliding, Session = pkg.TumblingWindow, pkg.SlidingWindow, pkg.SessionWindow
T = pkg.WindowMeasure.Time


def c4(batch, steps, keys, dev):
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    op = pkg.KeyedSlicingWindowOperator(device=0)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1)
    op.addWindowAssigner(Sliding(T, 60_000, 1_000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    bufs = []
    for s in range(steps):
        k = torch.randint(0, keys, (batch,), device=dev, dtype=torch.int32, generator=g)
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        bufs.append((k, base + s * 1000, v, s * 1000 + (batch - 1) // rate))
    torch.cuda.synchronize()
    times = []
    rows = 0
    for k, ts, v, wm in bufs:
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(wm)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        rows += n
        import numpy as np
        g = op._l.scotty_debug_dump
        g.restype, g.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
        buf = np.zeros(1 << 20, dtype=np.int64)
        k = g(op._h, 0, buf.ctypes.data, len(buf))
        S = int(buf[0])
        print("  slices", S, "tStart head..", buf[1:1 + min(S, 8)].tolist(), "tail part", buf[1 + 7 * S:k].tolist()[:30],
              flush=True)
    return times, rows, op.keyCount()


def c3(batch, steps, dev, ooo=0.2, delay=500):
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    op = pkg.SlicingWindowOperator(device=0)
    op.addWindowFunction(pkg.AGG_MIN_I32)
    op.addWindowFunction(pkg.AGG_MAX_I32)
    op.setMaxLateness(2 * delay)
    op.addWindowAssigner(Sliding(T, 60_000, 60))
    op.addWindowAssigner(Session(T, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    bufs = []
    for s in range(steps):
        ts = base + s * 1000 + 1000
        late = torch.rand(batch, device=dev, generator=g) < ooo
        d = torch.randint(1, delay + 1, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=1), ts)
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        bufs.append((ts.contiguous(), v, s * 1000 + 1000 + (batch - 1) // rate - delay))
    torch.cuda.synchronize()
    times = []
    rows = 0
    import ctypes
    f = op._l.scotty_debug_stat
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]
    for ts, v, wm in bufs:
        t0 = time.perf_counter()
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        t1 = time.perf_counter()
        n, _ = op.processWatermarkDevice(wm)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        print("step push %.1f ms, wm %.1f ms, events %d rounds %d" % ((t1 - t0) * 1e3, (time.perf_counter() - t1) * 1e3,
                                                                    f(op._h, 0), f(op._h, 1)), flush=True)
        rows += n
        import numpy as np
        g = op._l.scotty_debug_dump
        g.restype, g.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
        buf = np.zeros(1 << 20, dtype=np.int64)
        k = g(op._h, 0, buf.ctypes.data, len(buf))
        S = int(buf[0])
        print("  slices", S, "tStart head..", buf[1:1 + min(S, 8)].tolist(), "tail part", buf[1 + 7 * S:k].tolist()[:30],
              flush=True)
    return times, rows


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4-batch", type=int, default=1 << 24)
    ap.add_argument("--c4-keys", type=int, default=1 << 20)
    ap.add_argument("--c3-batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--which", default="c3,c4")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    if "c4" in a.which:
        t, rows, nk = c4(a.c4_batch, a.steps, a.c4_keys, dev)
        out["c4"] = {"batch": a.c4_batch, "keys": nk, "step_ms": [round(x * 1e3, 3) for x in t], "rows": rows,
                     "tuples_per_s_steady": a.c4_batch / (sum(t[1:]) / max(1, len(t) - 1))}
        print(json.dumps(out["c4"]), flush=True)
    if "c3" in a.which:
        t, rows = c3(a.c3_batch, a.steps, dev)
        out["c3"] = {"batch": a.c3_batch, "step_ms": [round(x * 1e3, 3) for x in t], "rows": rows,
                     "tuples_per_s_steady": a.c3_batch / (sum(t[1:]) / max(1, len(t) - 1))}
        print(json.dumps(out["c3"]), flush=True)
