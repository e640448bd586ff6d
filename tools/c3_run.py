"""Runs only bench.py's C3 leg (extra_c3) and prints its JSON: the command profiled by tools/gpu_c3q.sh."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    bench = importlib.import_module("bench")
    pkg = importlib.import_module("scotty-window-processor_amd")
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    r = bench.extra_c3(pkg, torch.device("cuda", 0), 1 << 26, steps)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
