#!/bin/bash
# round 3: quiet commit split into scan / multi-workgroup edges / commit, 64-ary slice searches in the exact
# watermark: exact + keyed suites, then the C3 leg (commit stamps) and its per-step kernel breakdown
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03q
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_keyed_grid.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03q/tests.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03q/tests.log | tail -6; exit 1; }
tail -1 gpurun_out/r03q/tests.log
SCOTTY_XQ_PROF=1 timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03q/c3.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03q/c3.log; exit 1; }
grep "xq commit" gpurun_out/r03q/c3.log | tail -4
grep '^{' gpurun_out/r03q/c3.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('c3', round(d['ms_per_step'],4), d['ms_per_step_each'], 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03q/c3prof -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/r03q/c3_run.log 2>&1 || { echo c3_prof_failed; tail -20 gpurun_out/r03q/c3_run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/r03q/c3prof/run_kernel_trace.csv > gpurun_out/r03q/c3_steps.txt
head -40 gpurun_out/r03q/c3_steps.txt
