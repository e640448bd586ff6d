#!/bin/bash
# round 3: keyed lane watermark computes MIN / MAX windows in the emit kernel (scan of each window's contained run):
# keyed + exact suites, then the C4 leg with SUM and with MIN + MAX
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03y
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed_grid.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03y/tests.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03y/tests.log | tail -6; exit 1; }
tail -1 gpurun_out/r03y/tests.log
for v in sum minmax; do
  timeout -k 10 300 python3 -u tools/c4_run.py 6 $v > gpurun_out/r03y/c4_$v.log 2>&1 || { echo c4_failed $v; tail -5 gpurun_out/r03y/c4_$v.log; exit 1; }
  grep '^{' gpurun_out/r03y/c4_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('C4 $v', round(d['value']/1e9,2), 'ms', round(d['ms_per_step'],4), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
done
