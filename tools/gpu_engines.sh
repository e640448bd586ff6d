#!/bin/bash
# Exact / keyed / count engines: parity, then the C3 / C4 / C5 / C5t bench legs.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_exact.py tests/test_golden.py tests/test_gpu_count.py tests/test_gpu_keyed_grid.py -x -q --timeout 300 --timeout-method thread > gpurun_out/engine_tests.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/engine_tests.log; exit 1; }
tail -1 gpurun_out/engine_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --only c3,c4,c5,c5t --steps 5 --warmup 2 > gpurun_out/bench_engines.log 2>&1 || { echo bench_failed; tail -10 gpurun_out/bench_engines.log; exit 1; }
python3 -c "
import json; r=json.loads([l for l in open('gpurun_out/bench_engines.log') if l.startswith('{')][-1])
for k,v in r['extra'].items(): print(k, round(v['value']/1e9,2), 'G/s', round(v['ms_per_step'],3), 'ms')"
echo all_ok
