#!/bin/bash
# round 4: keyed MIN/MAX block summaries -- parity, then the C4 watermark with MIN/MAX vs SUM
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed_minmax.py tests/test_gpu_exact.py -k "keyed" -x -v --timeout 400 --timeout-method thread > gpurun_out/r04c/tests.log 2>&1 || { echo tests_failed; grep -E "PASS|FAIL|Error|assert" gpurun_out/r04c/tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r04c/tests.log | tail -2
timeout -k 10 300 python -u tools/c4_run.py 5 minmax > gpurun_out/r04c/c4_minmax.json 2> gpurun_out/r04c/c4_minmax.err || { echo c4mm_failed; tail -20 gpurun_out/r04c/c4_minmax.err; exit 1; }
timeout -k 10 300 python -u tools/c4_run.py 5 > gpurun_out/r04c/c4_sum.json 2> gpurun_out/r04c/c4_sum.err || { echo c4_failed; tail -20 gpurun_out/r04c/c4_sum.err; exit 1; }
python3 - <<'PY'
import json
for n in ("c4_minmax", "c4_sum"):
    r = json.loads(open("gpurun_out/r04c/%s.json" % n).read().strip().splitlines()[-1])
    print(n, "G tuples/s %.1f" % (r["value"] / 1e9), "ms/step %.3f" % r["ms_per_step"],
          {k: round(v, 3) for k, v in r["roofline"]["device_ms_per_step_by_class"].items()})
PY
