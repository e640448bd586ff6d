"""C4 (keyed, 1M keys) at several per-step batch sizes: prints one JSON line per size (GPU box tool)."""
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
# args: log2 batch sizes and key=value tune knobs, e.g. `c4_sweep.py 26 keyed_grid_variant=0`
sizes = [int(x) for x in sys.argv[1:] if "=" not in x] or [24, 25, 26]
tune = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[1:] if "=" in kv)
for lg in sizes:
    r = bench.extra_c4(pkg, dev, 1 << lg, 1 << 20, 5, tune=tune)
    r["log2_batch"] = lg
    r["tune"] = tune
    print(json.dumps(r), flush=True)
    torch.cuda.empty_cache()
