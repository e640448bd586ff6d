#!/bin/bash
# Grid path: parity (random configs, JUnit goldens, golden fixtures, host ingest, sharding), then C2 + C2s bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_ingest.py tests/test_gpu_shard.py -x -q --timeout 250 --timeout-method thread > gpurun_out/grid_tests.log 2>&1 || { echo grid_tests_failed; tail -40 gpurun_out/grid_tests.log; exit 1; }
tail -1 gpurun_out/grid_tests.log
timeout -k 10 300 python -u bench.py --only c2s --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { echo bench_failed; tail -10 gpurun_out/bench_c2.log; exit 1; }
python3 -c "
import json; r=json.loads([l for l in open('gpurun_out/bench_c2.log') if l.startswith('{')][-1])
print('C2', round(r['value']/1e9,1), 'G/s', round(r['ms_per_step'],4), 'ms frac', round(r['roofline']['frac'],3), 'frac_step', round(r['roofline']['frac_step'],3), r['roofline']['device_ms_per_step_by_class'])
c=r['extra']['c2s']; print('C2s', round(c['value']/1e9,1), 'G/s', round(c['ms_per_step'],4), 'ms frac', round(c['roofline']['frac'],3), 'frac_step', round(c['roofline']['frac_step'],3), c['roofline']['device_ms_per_step_by_class'])"
echo all_ok
