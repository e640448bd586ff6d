#!/bin/bash
# round 3: grid watermark rows written straight into host-mapped memory (no publish launch), ambiguous edge candidates
# listed in LDS in the grid commit: grid-path suites, the headline bench line, and the keyed watermark's MIN/MAX
# assembly against SUM (C4 leg with MIN_I32 + MAX_I32)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest.py tests/test_gpu_shard.py tests/test_gpu_count.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03w/tests.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03w/tests.log | tail -6; exit 1; }
tail -1 gpurun_out/r03w/tests.log
timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline > gpurun_out/r03w/c2.json 2> gpurun_out/r03w/c2.log || { echo c2_failed; tail -5 gpurun_out/r03w/c2.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03w/c2.json')); r=d['roofline']
print('C2', round(d['value']/1e9,1), 'ms', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), 'frac_step', round(r['frac_step'],3), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
for v in sum minmax; do
  timeout -k 10 300 python3 -u tools/c4_run.py 6 $v > gpurun_out/r03w/c4_$v.log 2>&1 || { echo c4_failed $v; tail -5 gpurun_out/r03w/c4_$v.log; exit 1; }
  grep '^{' gpurun_out/r03w/c4_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('C4 $v', round(d['value']/1e9,2), 'ms', round(d['ms_per_step'],4), json.dumps({k: round(v,4) for k,v in r['device_ms_per_step_by_class'].items()}))"
done
