"""Interleaved same-box A/B of scotty_tune knobs on the C3 leg (bench.extra_c3: sliding + session windows, MIN / MAX,
20 % out of order, the exact engine's quiet pass): `python tools/ab_c3.py '{}' '{"quiet_ingest_mode": 23}'` runs each
knob set in turn, 2 rounds, one JSON line per run (wall ms per step, the quiet ingest's average launch).  GPU tool."""
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
tunes = [json.loads(x) for x in sys.argv[1:]] or [{}]
for rep in range(2):
    for t in tunes:
        r = bench.extra_c3(pkg, dev, 1 << 26, 10, tune=t)
        roof = r.get("roofline", {})
        print(json.dumps({"tune": t, "rep": rep, "ms_per_step": r["ms_per_step"], "each": r["ms_per_step_each"],
                          "ingest_ms": roof.get("avg_launch_ms"), "frac": roof.get("frac")}), flush=True)
        torch.cuda.empty_cache()
