"""Events and apply segments per push of the C3 leg (exact batch path): scotty_debug_stat 0 / 1 after each push."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("scotty-window-processor_amd")


def main():
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
    t72 = None
    for s in range(75):
        t_begin = s * 1000 + 1000 + (s // 10) * 1500
        ts = base + t_begin
        late = torch.rand(batch, device=dev, generator=g) < 0.2
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=t_begin - 500), ts).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)  # the operator's stream does not order after torch's
        if s == 73:
            os.environ["SCOTTY_XB_PROF"] = "1"  # the engine prints clock stamps of the event pass (stderr)
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        op.sync()
        os.environ.pop("SCOTTY_XB_PROF", None)
        ev, seg = op._debug_stat(0), op._debug_stat(1)
        n, _ = op.processWatermarkDevice(t_begin + (batch - 1) // rate - 500)
        if s >= 55:
            print("step %d events %d segments %d slices %d rows %d" % (s, ev, seg, op.sliceCount(), n), flush=True)


if __name__ == "__main__":
    main()
