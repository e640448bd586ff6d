"""C4s only (bench.py extra_c4s: keyed SessionWindow + SlidingWindow, 1 M keys, 2^26 tuples per step), for rocprofv3
kernel-trace / PMC passes over the keyed-session kernels without the other legs.

  python tools/c4s_probe.py [--steps 4] [--warm 6] [--keys 1048576] [--tune key=value ...]
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warm", type=int, default=6)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=1 << 26)
    ap.add_argument("--tune", nargs="*", default=[])
    args = ap.parse_args()
    import torch
    import bench
    pkg = importlib.import_module("scotty-window-processor_amd")
    tune = {k: int(v) for k, v in (x.split("=") for x in args.tune)}
    r = bench.extra_c4s(pkg, torch.device("cuda", 0), args.batch, args.keys, steps=args.steps, warm=args.warm,
                        tune=tune or None)
    roof = r.pop("roofline", {})
    r["device_ms_per_step_by_class"] = roof.get("device_ms_per_step_by_class")
    print(json.dumps(r))


if __name__ == "__main__":
    main()
