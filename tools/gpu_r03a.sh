#!/bin/bash
# round 3: quiet-path parity (exact engine) + C3 bench leg
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread \
  -k "quiet or config3 or session or batch_parallel" > gpurun_out/r03a_tests.log 2>&1 || { tail -50 gpurun_out/r03a_tests.log; exit 1; }
tail -5 gpurun_out/r03a_tests.log
timeout -k 10 400 python -u bench.py --only c3 --no-cpu-baseline --steps 5 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.log || { tail -30 gpurun_out/r03a_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03a_bench.json"))
c3 = d["extra"]["c3"]
print(json.dumps({k: c3[k] for k in ("ms_per_step", "ms_per_step_each", "quiet_steps", "event_exact_steps", "value")}))
print(json.dumps(c3["roofline"]))
PY
