"""Wall-clock phases of the C5t leg (SURVEY C5 on the count path): push vs watermark per step, synchronised."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import importlib
    pkg = importlib.import_module("scotty-window-processor_amd")
    dev = torch.device("cuda", 0)
    batch = 1 << 26
    op = pkg.SlicingWindowOperator(device=0)
    op.tune("count_path", 1)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Count, 1000))
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60000, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for s in range(8):
        ts = base + s * batch
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n, _ = op.processWatermarkDevice((s + 1) * batch - 1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("step %d: push %.3f ms (time-edge host step %d us), watermark %.3f ms, %d windows, time edges %d" %
              (s, 1e3 * (t1 - t0), op._debug_stat(7), 1e3 * (t2 - t1), n, op._debug_stat(6)), flush=True)


if __name__ == "__main__":
    main()
