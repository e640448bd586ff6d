"""A/B of ingest-kernel variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

Runs the C2 bench workload; before each push selects a variant via the undeclared scotty_tune hook and
reads the HIP-event ingest time of that push.  Prints median/min per variant.
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
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("scotty-window-processor_amd")
    L = pkg.lib()
    L.scotty_tune.restype = ctypes.c_int
    L.scotty_tune.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
    modes = [int(m) for m in args.modes.split(",")]
    B = args.batch
    rate = B // 1000
    dev = torch.device("cuda", 0)
    op = pkg.SlicingWindowOperator()
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for s in pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10):
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    base = torch.arange(B, device=dev, dtype=torch.int64) // rate
    vals = torch.randint(-2**31, 2**31, (B,), device=dev, dtype=torch.int32)
    nb = (args.rounds + 1) * len(modes)
    bufs = [base + k * 1000 for k in range(nb)]   # pre-generated, like bench.py (no dirty lines at push time)
    torch.cuda.synchronize(dev)
    op.enableTiming(True)
    res = {m: [] for m in modes}
    step = 0
    for r in range(args.rounds + 1):
        for m in modes:
            ts = bufs[step]
            L.scotty_tune(op._h, b"ingest_mode", m)
            before = op.ingestTiming()[0]
            op.processElementsDevice(ts.data_ptr(), vals.data_ptr(), B)
            op.processWatermarkRaw(step * 1000 + 999)
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
