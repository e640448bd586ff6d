#!/bin/bash
# round 3: parity after (ingest step maxima, grouped drain, quiet commit narrowing, chunked event prefix, keyed
# scatter variants), then C3 ingest-mode A/B and the C4 keyed-variant A/B
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r03h/tests.log 2>&1 || { tail -30 gpurun_out/r03h/tests.log; exit 1; }
tail -2 gpurun_out/r03h/tests.log
SCOTTY_TEST_KG_VARIANT=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_keyed_grid.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03h/keyed_grid_v4.log 2>&1 || { tail -40 gpurun_out/r03h/keyed_grid_v4.log; exit 1; }
tail -1 gpurun_out/r03h/keyed_grid_v4.log
for m in 6 14 2; do
  SCOTTY_INGEST_MODE=$m SCOTTY_XQ_PROF=1 timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03h/c3_mode$m.log 2>&1 || { echo c3_failed_$m; tail -20 gpurun_out/r03h/c3_mode$m.log; exit 1; }
  echo "mode $m"; grep "xq commit" gpurun_out/r03h/c3_mode$m.log | tail -3
  grep '^{' gpurun_out/r03h/c3_mode$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(round(d['ms_per_step'],4), d['ms_per_step_each'], 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}), 'tail_commits', d.get('event_prefix_then_quiet_steps'))"
done
timeout -k 10 500 python3 -u tools/c4_ab.py 1,4,5,6 6 > gpurun_out/r03h/c4_ab.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/r03h/c4_ab.log; exit 1; }
grep variant gpurun_out/r03h/c4_ab.log
