#!/bin/bash
# round 3: event-exact rounds chained on the device, chain length predicted from the last multi-round push (the
# exact suite runs in the full -m gpu pass): the C3 leg and its pause-step breakdown
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03aa
timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03aa/c3.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03aa/c3.log; exit 1; }
grep '^{' gpurun_out/r03aa/c3.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d["roofline"]; print("c3", round(d["ms_per_step"],4), d["ms_per_step_each"], d.get("events_rounds_each")[-1], json.dumps({k: round(v,4) for k,v in r["device_ms_per_step_by_class"].items()}))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03aa/c3prof -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/r03aa/c3_run.log 2>&1 || { echo c3_prof_failed; tail -20 gpurun_out/r03aa/c3_run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/r03aa/c3prof/run_kernel_trace.csv > gpurun_out/r03aa/c3_steps.txt
tail -16 gpurun_out/r03aa/c3_steps.txt
