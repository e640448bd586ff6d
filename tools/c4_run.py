"""Runs only bench.py's C4 leg (extra_c4: 2^26 tuples, 2^20 keys per step) and prints its JSON: the command profiled
by the round-3 C4 trace scripts."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    bench = importlib.import_module("bench")
    pkg = importlib.import_module("scotty-window-processor_amd")
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    aggs = None
    if len(sys.argv) > 2 and sys.argv[2] == "minmax":  # the keyed watermark's MIN/MAX assembly vs the SUM prefix path
        aggs = (pkg.AGG_MIN_I32, pkg.AGG_MAX_I32)
    r = bench.extra_c4(pkg, torch.device("cuda", 0), bench.C4_BATCH, 1 << 20, steps, aggs=aggs)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
