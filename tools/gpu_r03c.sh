#!/bin/bash
# round 3: keyed engine after the key-interleaved slice store -- keyed parity suites + C4 leg with device roofline
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py tests/test_gpu_exact.py -k "keyed" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03c_keyed.log 2>&1 || { tail -40 gpurun_out/r03c_keyed.log; exit 1; }
tail -3 gpurun_out/r03c_keyed.log
timeout -k 10 400 python -u bench.py --only c4 --no-cpu-baseline --steps 8 > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.log || { tail -30 gpurun_out/r03c_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03c_bench.json"))
x = d["extra"]["c4"]
print(json.dumps({a: x.get(a) for a in ("ms_per_step", "value", "roofline")}))
PY
