#!/bin/bash
# round 4: exact-engine block summaries + LDS commit -- parity, then C2 / C3 bench legs
set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 1000 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r04d/tests.log 2>&1 || { echo tests_failed; grep -E "PASS|FAIL|Error|assert" gpurun_out/r04d/tests.log | tail -30; exit 1; }
tail -2 gpurun_out/r04d/tests.log
timeout -k 10 400 python -u bench.py --only c3 --no-cpu-baseline > gpurun_out/r04d/bench.json 2> gpurun_out/r04d/bench.err || { echo bench_failed; tail -20 gpurun_out/r04d/bench.err; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r04d/bench.json").read().strip().splitlines()[-1])
print("C2 G/s %.1f ms %.4f frac %.3f frac_step %.3f" % (r["value"] / 1e9, r["ms_per_step"], r["roofline"]["frac"], r["roofline"]["frac_step"]),
      {k: round(v * 1e3, 1) for k, v in r["roofline"]["device_ms_per_step_by_class"].items()})
c3 = r["extra"]["c3"]
print("C3 G/s %.1f ms %.3f" % (c3["value"] / 1e9, c3["ms_per_step"]), c3["ms_per_step_each"],
      {k: round(v * 1e3, 1) for k, v in c3["roofline"]["device_ms_per_step_by_class"].items()})
PY
