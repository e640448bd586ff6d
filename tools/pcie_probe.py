"""PCIe H2D probe (PCIe-inclusive leg): what the box's link delivers to plain copies, beside the leg.
Pinned 512 MiB host -> HBM: one hipMemcpyAsync; two halves on two streams at once; pageable; and D2H.  Prints one
JSON line.  Placement: the GPU's NUMA node and this process's CPU affinity are recorded (bench.py gpu_numa_node)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rate(fn, nbytes, reps=8):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    dev = torch.device("cuda", 0)
    nb = 512 << 20
    h = torch.empty(nb, dtype=torch.uint8).pin_memory()
    hp = torch.empty(nb, dtype=torch.uint8)
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    h.fill_(1)
    hp.fill_(1)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    half = nb // 2

    def two():
        with torch.cuda.stream(s1):
            d[:half].copy_(h[:half], non_blocking=True)
        with torch.cuda.stream(s2):
            d[half:].copy_(h[half:], non_blocking=True)

    out = {"bytes": nb,
           "h2d_pinned_GBs": rate(lambda: d.copy_(h, non_blocking=True), nb),
           "h2d_pinned_two_streams_GBs": rate(two, nb),
           "h2d_pageable_GBs": rate(lambda: d.copy_(hp), nb, reps=3),
           "d2h_pinned_GBs": rate(lambda: h.copy_(d, non_blocking=True), nb)}
    try:
        import bench
        out["gpu_numa_node"] = bench.gpu_numa_node(0)
    except Exception as e:  # placement is informative only
        out["gpu_numa_node"] = repr(e)
    out["affinity_cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
