"""C4 leg with the push and the watermark timed separately (host wall clock, synchronised), to split the step's
wall time from its device time."""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("scotty-window-processor_amd")


def main():
    dev = torch.device("cuda", 0)
    batch = 1 << 26
    rate = batch // 1000
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    op = pkg.KeyedSlicingWindowOperator(device=0)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 1_000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    tp, tw = [], []
    for s in range(70):
        k = torch.randint(0, 1 << 20, (batch,), device=dev, dtype=torch.int32, generator=g)
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        ts = base + s * 1000
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        op.sync()
        t1 = time.perf_counter()
        op.processWatermarkDevice(s * 1000 + (batch - 1) // rate)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        if s >= 62:
            tp.append(t1 - t0)
            tw.append(t2 - t1)
            print("step %d push %.3f ms  watermark %.3f ms  path %d deferred %d" % (
                s, 1e3 * (t1 - t0), 1e3 * (t2 - t1), op._debug_stat(2), op._debug_stat(3)), flush=True)
    print("median push %.3f ms, watermark %.3f ms" % (1e3 * np.median(tp), 1e3 * np.median(tw)))


if __name__ == "__main__":
    main()
