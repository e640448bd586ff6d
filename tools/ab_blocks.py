"""Ingest launch width A/B on the C2 workload (interleaved rounds in one process): HIP-event ingest time per
scotty_tune("ingest_blocks", B) value."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("scotty-window-processor_amd")


def main():
    blocks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1024,2048,512,1536").split(",")]
    B = 1 << 27
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
    res = {b: [] for b in blocks}
    step = 0
    op.enableTiming(True)
    for rnd in range(8):
        for b in blocks:
            op.tune("ingest_blocks", b)
            ts = base + step * 1000
            torch.cuda.synchronize()
            t0 = op.ingestTiming()
            op.processElementsDevice(ts.data_ptr(), vals.data_ptr(), B)
            op.processWatermarkRaw(step * 1000 + 999)
            t1 = op.ingestTiming()
            if rnd > 0:
                res[b].append(t1[0] - t0[0])
            step += 1
    for b in blocks:
        x = np.array(res[b])
        print("ingest_blocks %5d: median %.4f ms  min %.4f ms  -> %.2f TB/s" % (b, np.median(x), x.min(),
                                                                          12 * B / np.median(x) / 1e9))


if __name__ == "__main__":
    main()
