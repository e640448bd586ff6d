#!/bin/bash
# round 4: streaming ingest variant -- grid-path parity, then the C2 line with the C1 / C2s legs
set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "not c3" -x -q --timeout 400 --timeout-method thread > gpurun_out/r04g/tests.log 2>&1 || { echo tests_failed; grep -E "PASS|FAIL|Error|assert" gpurun_out/r04g/tests.log | tail -30; exit 1; }
tail -2 gpurun_out/r04g/tests.log
timeout -k 10 400 python -u bench.py --only c1,c2s --no-cpu-baseline > gpurun_out/r04g/bench.json 2> gpurun_out/r04g/bench.err || { echo bench_failed; tail -20 gpurun_out/r04g/bench.err; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r04g/bench.json").read().strip().splitlines()[-1])
print("C2 G/s %.1f ms %.4f frac %.3f frac_step %.3f" % (r["value"] / 1e9, r["ms_per_step"], r["roofline"]["frac"], r["roofline"]["frac_step"]),
      {k: round(v * 1e3, 1) for k, v in r["roofline"]["device_ms_per_step_by_class"].items()})
for leg in ("c1", "c2s"):
    c = r["extra"][leg]
    print(leg, "G/s %.1f ms %.4f frac %.3f" % (c["value"] / 1e9, c["ms_per_step"], c["roofline"]["frac"]),
          {k: round(v * 1e3, 1) for k, v in c["roofline"]["device_ms_per_step_by_class"].items()})
PY
