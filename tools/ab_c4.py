"""Interleaved same-box A/B of the keyed sort-free path's kernel variants on C4 (2^26 tuples, 2^20 keys, SUM_I32):
`python tools/ab_c4.py 0 1` runs variant 0, variant 1, variant 0, variant 1, ... (3 rounds), one JSON line per run with
the wall ms per step and the per-class device ms (HIP events).  GPU box tool."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

pkg = importlib.import_module("scotty-window-processor_amd")
dev = torch.device("cuda", 0)
variants = [int(x) for x in sys.argv[1:]] or [0, 1]
for rep in range(3):
    for v in variants:
        r = bench.extra_c4(pkg, dev, 1 << 26, 1 << 20, 5, tune={"keyed_grid_variant": v})
        roof = r.get("roofline", {})
        print(json.dumps({"variant": v, "rep": rep, "ms_per_step": r.get("ms_per_step"), "value": r.get("value"),
                          "device_ms_by_class": roof.get("device_ms_per_step_by_class"),
                          "data_pass_ms": roof.get("avg_launch_ms")}), flush=True)
        torch.cuda.empty_cache()
