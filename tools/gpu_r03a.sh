#!/bin/bash
# round 3: quiet-path parity (exact engine) + C3 bench leg
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -v -s --timeout 500 --timeout-method thread \
  -k "config3_full_size" > gpurun_out/r03a_full.log 2>&1 || { tail -40 gpurun_out/r03a_full.log; exit 1; }
tail -12 gpurun_out/r03a_full.log
timeout -k 10 400 python -u bench.py --only c3 --no-cpu-baseline --steps 5 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.log || { tail -30 gpurun_out/r03a_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03a_bench.json"))
c3 = d["extra"]["c3"]
print(json.dumps({k: c3[k] for k in ("ms_per_step", "ms_per_step_each", "quiet_steps", "event_exact_steps", "value")}))
print(json.dumps(c3["roofline"]))
PY
