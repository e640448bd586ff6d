"""Wall-clock phases of the C3 leg (exact batch path): push vs watermark per step, events and apply segments of
each push (scotty_debug_stat 0 / 1).  Same stream as bench.py extra_c3."""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    pkg = importlib.import_module("scotty-window-processor_amd")
    dev = torch.device("cuda", 0)
    batch = 1 << 26
    rate = batch // 1000
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    op = pkg.SlicingWindowOperator(device=0)
    op.addWindowFunction(pkg.AGG_MIN_I32)
    op.addWindowFunction(pkg.AGG_MAX_I32)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 60))
    op.addWindowAssigner(pkg.SessionWindow(pkg.WindowMeasure.Time, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    for s in range(int(sys.argv[1]) if len(sys.argv) > 1 else 70):
        t_begin = s * 1000 + 1000 + (s // 10) * 1500
        ts = base + t_begin
        late = torch.rand(batch, device=dev, generator=g) < 0.2
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=t_begin - 500), ts).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n, _ = op.processWatermarkDevice(t_begin + (batch - 1) // rate - 500)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if s >= 55:
            print("step %d: push %.3f ms (events %d, segments %d), watermark %.3f ms, %d windows, %d slices" %
                  (s, 1e3 * (t1 - t0), op._debug_stat(0), op._debug_stat(1), 1e3 * (t2 - t1), n, op.sliceCount()),
                  flush=True)


if __name__ == "__main__":
    main()
