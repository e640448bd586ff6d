"""C4 leg at a given key count (argv[1], default 2^20) and keyed-grid variant (argv[2], default 1): the bucket count of the
sort-free partition follows the key table (2 x keys positions, 1024 per bucket), so this isolates how the partition
scatter's run length (8192-tuple tiles / buckets records per bucket run) drives its rate.  One JSON line.  GPU tool,
run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

pkg = importlib.import_module("scotty-window-processor_amd")
keys = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 1
r = bench.extra_c4(pkg, torch.device("cuda", 0), 1 << 26, keys, 5, tune={"keyed_grid_variant": variant})
roof = r.get("roofline", {})
print(json.dumps({"keys": keys, "variant": variant, "ms_per_step": r["ms_per_step"], "value": r["value"],
                  "device_ms_by_class": roof.get("device_ms_per_step_by_class")}), flush=True)
