"""Standalone timing of the exact engine's bench legs (bench.py extra_c3 / extra_c4) for rocprofv3 runs:
BASELINE configs[2] (C3, non-keyed sliding+session, 20% OOO, MIN/MAX) and configs[3] (C4, keyed sliding
60s/1s SUM).  Inputs resident in HBM; results stay in HBM.

    python tools/perf_exact.py c4 --keys 1048576 --batch 16777216 --steps 5 [--wave]
"""
import argparse
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("scotty-window-processor_amd")
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["c2s", "c3", "c4", "c5"])
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--wave", action="store_true", help="C4: wavefront-per-key replay (tune keyed_lane 0)")
    ap.add_argument("--ooo", type=float, default=0.2, help="C2s: out-of-order fraction")
    ap.add_argument("--tune", action="append", default=[], help="C2s: scotty_tune key=value (repeatable)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.which == "c2s":
        tune = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.tune}
        r = bench.extra_c2s(pkg, dev, args.batch or (1 << 27), args.steps, tune=tune, ooo=args.ooo)
    elif args.which == "c5":
        r = bench.extra_c5(pkg, dev, args.batch or (1 << 27), args.steps)
    elif args.which == "c3":
        r = bench.extra_c3(pkg, dev, args.batch or (1 << 26), args.steps)
    else:
        r = bench.extra_c4(pkg, dev, args.batch or (1 << 24), args.keys, args.steps, lane=not args.wave)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
