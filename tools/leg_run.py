"""Runs ONE secondary leg of bench.py (c1, c2s, c3, c4, c5, c5t) in its own process and prints its JSON: the command
each per-leg rocprofv3 run profiles (tools/gpu_r03_final.sh), so every leg's kernel stats come from a trace of that
leg alone.  The headline C2 leg alone is `bench.py --no-extra --no-cpu-baseline`."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    bench = importlib.import_module("bench")
    pkg = importlib.import_module("scotty-window-processor_amd")
    leg = sys.argv[1]
    dev = torch.device("cuda", 0)
    run = {"c1": lambda: bench.extra_c1(pkg, dev, 1 << 26, 5),
           "c2s": lambda: bench.extra_c2s(pkg, dev, 1 << 27, 5),
           "c3": lambda: bench.extra_c3(pkg, dev, 1 << 26, 10),
           "c4": lambda: bench.extra_c4(pkg, dev, bench.C4_BATCH, 1 << 20, 5),
           "c5": lambda: bench.extra_c5(pkg, dev, 1 << 27, 5),
           "c5t": lambda: bench.extra_c5t(pkg, dev, 1 << 26, 5)}[leg]
    r = run()
    print(json.dumps({"leg": leg, **r}), flush=True)


if __name__ == "__main__":
    main()
