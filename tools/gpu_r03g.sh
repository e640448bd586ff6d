#!/bin/bash
# round 3: exact engine tests verbose (segment continuation), then the C3 leg with commit phase stamps and trace
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03g
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread \
  -s > gpurun_out/r03g/tests.log 2>&1 || { tail -60 gpurun_out/r03g/tests.log; exit 1; }
tail -2 gpurun_out/r03g/tests.log
SCOTTY_XQ_PROF=1 timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03g/c3_prof.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03g/c3_prof.log; exit 1; }
grep "xq commit" gpurun_out/r03g/c3_prof.log | tail -12
grep '^{' gpurun_out/r03g/c3_prof.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['ms_per_step'], d['ms_per_step_each'], json.dumps(d['roofline']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03g/c3 -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/r03g/c3_run.log 2>&1 || { echo c3_prof_failed; tail -20 gpurun_out/r03g/c3_run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/r03g/c3/run_kernel_trace.csv > gpurun_out/r03g/c3_steps.txt
cat gpurun_out/r03g/c3_steps.txt
