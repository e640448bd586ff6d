#!/bin/bash
# round 3: keyed suite on the pipelined scatter (variant 4), C3 ingest-mode A/B (6 default, 14 grouped-count drain,
# 2 no deferred queue), C4 keyed-variant A/B (1 default, 4 pipelined scatter, 5/6 + bucket loads 4/8 deep)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03k
SCOTTY_TEST_KG_VARIANT=5 timeout -k 10 400 python -u -m pytest tests/test_gpu_keyed_grid.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03k/keyed_grid_v5.log 2>&1 || { tail -40 gpurun_out/r03k/keyed_grid_v5.log; exit 1; }
tail -1 gpurun_out/r03k/keyed_grid_v5.log
for m in 6 14 2; do
  SCOTTY_INGEST_MODE=$m timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03k/c3_mode$m.log 2>&1 || { echo c3_failed_$m; tail -20 gpurun_out/r03k/c3_mode$m.log; exit 1; }
  echo "mode $m"
  grep '^{' gpurun_out/r03k/c3_mode$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(round(d['ms_per_step'],4), d['ms_per_step_each'], 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}), 'tail_commits', d.get('event_prefix_then_quiet_steps'))"
done
timeout -k 10 500 python3 -u tools/c4_ab.py 1,4,5,6 6 > gpurun_out/r03k/c4_ab.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/r03k/c4_ab.log; exit 1; }
grep variant gpurun_out/r03k/c4_ab.log
