#!/bin/bash
# round 3 re-entry: exact-engine GPU suite (incl. quiet path + full size) + C3 / C1 legs
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/r03b_exact.log 2>&1 || { tail -40 gpurun_out/r03b_exact.log; exit 1; }
tail -5 gpurun_out/r03b_exact.log
timeout -k 10 400 python -u bench.py --only c3,c1 --no-cpu-baseline --steps 10 > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.log || { tail -30 gpurun_out/r03b_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03b_bench.json"))
for k in ("c3", "c1"):
    x = d["extra"].get(k, {})
    print(k, json.dumps({a: x.get(a) for a in ("ms_per_step", "value", "quiet_steps", "event_exact_steps", "roofline")}))
PY
