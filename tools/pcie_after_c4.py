"""Does a plain pinned host->HBM copy slow down after the C4 leg ran in the same process?  (The PCIe-inclusive leg
measures 14.4 ms per step alone and 18-19 ms after C4: tools/gpu_r06_p17.sh / p18.)  Probe before, after C4, and
after C4 with every C4 object released (fresh pinned and device buffers each time); one JSON line."""
import gc
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from pcie_probe import rate  # noqa: E402


def probe(tag, out, extra_mib=0):
    # a size no earlier probe used and an emptied device cache: fresh pinned pages and a fresh device buffer (torch's
    # caching host allocator would otherwise hand back the block pinned before C4)
    nb = (512 + extra_mib) << 20
    dev = torch.device("cuda", 0)
    torch.cuda.empty_cache()
    h = torch.empty(nb, dtype=torch.uint8).pin_memory()
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    out[tag + "_h2d_pinned_GBs"] = rate(lambda: d.copy_(h, non_blocking=True), nb)
    out[tag + "_d2d_GBs"] = rate(lambda: d[: nb // 2].copy_(d[nb // 2:]), nb // 2)
    del h, d


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    pkg = importlib.import_module("scotty-window-processor_amd")
    out = {}
    sizes = pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10)
    leg = "--leg" in sys.argv  # the product's host-fed leg (bench.extra_pcie) before and after C4 as well
    probe("before", out)
    if leg:
        out["before_leg_pinned_ms"] = bench.extra_pcie(pkg, sizes, 1 << 26, 5)["pinned"]["ms_per_step"]
    r = bench.extra_c4(pkg, dev, bench.C4_BATCH, 1 << 20, 5, host_steps=5)
    out["c4_ms_per_step"] = r["ms_per_step"]
    probe("after_c4", out, 2)
    if leg:
        out["after_c4_leg_pinned_ms"] = bench.extra_pcie(pkg, sizes, 1 << 26, 5)["pinned"]["ms_per_step"]
    del r
    gc.collect()
    torch.cuda.empty_cache()
    probe("after_c4_released", out, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
