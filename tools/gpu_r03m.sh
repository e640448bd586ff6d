#!/bin/bash
# round 3: compact LDS window (32-bit tmax offsets, int32 min/max): parity, C3 modes, C2s, C1
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "quiet or config3 or session or parity" > gpurun_out/r03m/tests.log 2>&1 || { tail -30 gpurun_out/r03m/tests.log; exit 1; }
tail -1 gpurun_out/r03m/tests.log
for m in 6 7; do
  SCOTTY_INGEST_MODE=$m timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03m/c3_mode$m.log 2>&1 || { echo c3_failed_$m; tail -20 gpurun_out/r03m/c3_mode$m.log; exit 1; }
  grep '^{' gpurun_out/r03m/c3_mode$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('c3 mode $m', round(d['ms_per_step'],4), d['ms_per_step_each'], 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
done
for leg in c2s c1; do
  timeout -k 10 300 python3 -u tools/leg_run.py $leg > gpurun_out/r03m/$leg.log 2>&1 || { echo leg_failed_$leg; tail -20 gpurun_out/r03m/$leg.log; exit 1; }
  grep '^{' gpurun_out/r03m/$leg.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('$leg', round(d['ms_per_step'],4), 'G/s', round(d['value']/1e9,1), 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), 'frac_step', round(r['frac_step'],3))"
done
