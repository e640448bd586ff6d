"""A/B of ingest-kernel variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

Runs the C2 bench workload; before each push selects a variant ("mode" or "mode:blocks": scotty_tune ingest_mode and
ingest_blocks) and reads the HIP-event ingest time of that push.  Prints median/min per variant.
"""
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
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1 << 27)
    ap.add_argument("--c2s", action="store_true", help="C2s: 1000 sliding windows, 20%% of the tuples late by U[1,500] ms")
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("scotty-window-processor_amd")
    L = pkg.lib()
    L.scotty_tune.restype = ctypes.c_int
    L.scotty_tune.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
    modes = args.modes.split(",")
    B = args.batch
    rate = B // 1000
    dev = torch.device("cuda", 0)
    op = pkg.SlicingWindowOperator()
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    if args.c2s:
        bench = importlib.import_module("bench")
        op.setMaxLateness(1000)
        for size, slide in bench.c2s_windows(pkg):
            op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, size, slide))
    else:
        op.setMaxLateness(1)
        for s in pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10):
            op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    base = torch.arange(B, device=dev, dtype=torch.int64) // rate
    vals = torch.randint(-2**31, 2**31, (B,), device=dev, dtype=torch.int32)
    nb = (args.rounds + 1) * len(modes)
    g = torch.Generator(device=dev)
    g.manual_seed(5)

    def mk(k):
        ts = base + k * 1000 + 1000
        if args.c2s:
            late = torch.rand(B, device=dev, generator=g) < 0.2
            d = torch.randint(1, 501, (B,), device=dev, generator=g)
            ts = torch.where(late, torch.clamp(ts - d, min=1), ts).contiguous()
        return ts
    bufs = [mk(k) for k in range(nb)]   # pre-generated, like bench.py (no dirty lines at push time)
    torch.cuda.synchronize(dev)
    op.enableTiming(True)
    res = {m: [] for m in modes}
    step = 0
    for r in range(args.rounds + 1):
        for m in modes:
            ts = bufs[step]
            mm, _, blk = m.partition(":")
            L.scotty_tune(op._h, b"ingest_mode", int(mm))
            L.scotty_tune(op._h, b"ingest_blocks", int(blk) if blk else 256 * 4)
            before = op.ingestTiming()[0]
            op.processElementsDevice(ts.data_ptr(), vals.data_ptr(), B)
            op.processWatermarkRaw(step * 1000 + 1999 - (500 if args.c2s else 0))
            ms = op.ingestTiming()[0] - before
            if r > 0:
                res[m].append(ms)
            step += 1
    out = {}
    for m in modes:
        a = np.array(res[m])
        out[m] = {"median_ms": float(np.median(a)), "min_ms": float(a.min()),
                  "median_TBps": B * 12 / (np.median(a) * 1e-3) / 1e12}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
