#!/bin/bash
# round 3: quiet commit narrowed by the ingest's step maxima (retry without the unrolled verdict loads): exact suite,
# then the C3 leg with commit phase stamps
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03n
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03n/tests.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03n/tests.log | tail -4; exit 1; }
tail -1 gpurun_out/r03n/tests.log
SCOTTY_XQ_PROF=1 timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03n/c3.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03n/c3.log; exit 1; }
grep "xq commit" gpurun_out/r03n/c3.log | tail -4
grep '^{' gpurun_out/r03n/c3.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('c3', round(d['ms_per_step'],4), d['ms_per_step_each'], 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
