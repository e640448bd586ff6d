#!/bin/bash
# round 3: exact-engine allocations zero-filled (ordered before the operator's stream uses them); the exact suite
# that faulted in r03r (test_session_streams_match_oracle[11] after 61 tests), then the parity suite
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03s
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03s/tests_exact.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03s/tests_exact.log | tail -6; exit 1; }
tail -1 gpurun_out/r03s/tests_exact.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keyed_grid.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03s/tests_parity.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03s/tests_parity.log | tail -6; exit 1; }
tail -1 gpurun_out/r03s/tests_parity.log
timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03s/c3.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03s/c3.log; exit 1; }
grep '^{' gpurun_out/r03s/c3.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d["roofline"]; print("c3", round(d["ms_per_step"],4), d["ms_per_step_each"], d.get("events_rounds_each"), "ingest_ms", round(r["avg_launch_ms"],4), "frac", round(r["frac"],3), json.dumps({k: round(v,4) for k,v in r["device_ms_per_step_by_class"].items()}))'
