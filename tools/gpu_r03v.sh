#!/bin/bash
# round 3: count lookups of the watermark's aggregation range narrowed, 64-ary pending-edge search in the quiet prep:
# exact suite, C3 leg, then the headline C2 leg's per-step kernel breakdown
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03v/tests_exact.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03v/tests_exact.log | tail -6; exit 1; }
tail -1 gpurun_out/r03v/tests_exact.log
timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03v/c3.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03v/c3.log; exit 1; }
grep '^{' gpurun_out/r03v/c3.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d["roofline"]; print("c3", round(d["ms_per_step"],4), d["ms_per_step_each"], json.dumps({k: round(v,4) for k,v in r["device_ms_per_step_by_class"].items()}))'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03v/prof_c2 -o run --output-format csv -- python3 -u bench.py --no-extra --no-cpu-baseline > gpurun_out/r03v/prof_c2.log 2>&1 || { echo prof_failed c2; tail -5 gpurun_out/r03v/prof_c2.log; exit 1; }
python3 tools/trace_c3.py --marker ingest_kernel gpurun_out/r03v/prof_c2/run_kernel_trace.csv > gpurun_out/r03v/c2_steps.txt
cat gpurun_out/r03v/c2_steps.txt
