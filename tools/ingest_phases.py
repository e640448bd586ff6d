"""Phase split of the grid ingest kernel from its per-workgroup clock stamps (scotty_tune "ingest_stamps"): C2 or C2s
(--c2s) at the bench size, a few pushes, then for the last push the median over workgroups of (window ready - start),
(ranges done - window ready), (window flushed - ranges done) and the spread of the workgroups' start and end
stamps, in microseconds (s_memtime ticks / --ghz); and the commit kernel's phase split (commit_*: the ticks between
its stamps).  GPU box tool."""
import argparse
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2s", action="store_true")
    ap.add_argument("--mode", type=int, default=-1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--ghz", type=float, default=0.1, help="s_memtime ticks per ns (100 MHz constant clock: 0.1)")
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("scotty-window-processor_amd")
    bench = importlib.import_module("bench")
    L = pkg.lib()
    f = L.scotty_debug_ingest_stamps
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    fc = L.scotty_debug_commit_stamps
    fc.restype, fc.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p]
    B = 1 << 27
    rate = B // 1000
    dev = torch.device("cuda", 0)
    op = pkg.SlicingWindowOperator()
    op.tune("ingest_stamps", 1)
    if args.mode >= 0:
        op.tune("ingest_mode", args.mode)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    if args.c2s:
        op.setMaxLateness(1000)
        for size, slide in bench.c2s_windows(pkg):
            op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, size, slide))
    else:
        op.setMaxLateness(1)
        for s in pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10):
            op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    base = torch.arange(B, device=dev, dtype=torch.int64) // rate
    vals = torch.randint(-2**31, 2**31, (B,), device=dev, dtype=torch.int32)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    out = {}
    for k in range(args.steps):
        ts = base + k * 1000 + 1000
        if args.c2s:
            late = torch.rand(B, device=dev, generator=g) < 0.2
            d = torch.randint(1, 501, (B,), device=dev, generator=g)
            ts = torch.where(late, torch.clamp(ts - d, min=1), ts).contiguous()
        torch.cuda.synchronize(dev)
        op.processElementsDevice(ts.data_ptr(), vals.data_ptr(), B)
        op.processWatermarkRaw(k * 1000 + 1999 - (500 if args.c2s else 0))
        buf = np.zeros((8192, 4), dtype=np.int64)
        nb = f(op._h, buf.ctypes.data, 8192)
        st = buf[:nb]
        us = lambda x: float(x) / args.ghz / 1e3
        t0 = st[:, 0].min()
        out = {"step": k, "workgroups": int(nb),
               "prologue_us_median": us(np.median(st[:, 1] - st[:, 0])),
               "ranges_us_median": us(np.median(st[:, 2] - st[:, 1])),
               "flush_us_median": us(np.median(st[:, 3] - st[:, 2])),
               "flush_us_max": us(np.max(st[:, 3] - st[:, 2])),
               "start_spread_us": us(st[:, 0].max() - t0), "end_spread_us": us(st[:, 3].max() - st[:, 3].min()),
               "span_us": us(st[:, 3].max() - t0)}
        cb = np.zeros(8, dtype=np.int64)
        if fc(op._h, cb.ctypes.data) == 7:
            out["commit_ticks"] = [int(cb[i + 1] - cb[i]) for i in range(6)]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
