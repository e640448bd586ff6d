#!/bin/bash
# Sort-free keyed path: parity (new tests + the keyed exact-engine tests), then the C4 bench leg + rocprof.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py -x -v --timeout 300 --timeout-method thread > gpurun_out/kg_tests.log 2>&1 || { echo kg_tests_failed; tail -60 gpurun_out/kg_tests.log; exit 1; }
tail -3 gpurun_out/kg_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -k keyed -x -q --timeout 300 --timeout-method thread > gpurun_out/keyed_tests.log 2>&1 || { echo keyed_tests_failed; tail -60 gpurun_out/keyed_tests.log; exit 1; }
tail -2 gpurun_out/keyed_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --only c4 > gpurun_out/bench_c4.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench_c4.log; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1]); c=r['extra']['c4']; print('C4', c['value']/1e9, 'G t/s', c['ms_per_step'], 'ms/step')"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c4 > gpurun_out/prof_c4.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c4.log; exit 1; }
head -14 gpurun_out/prof_c4/run_kernel_stats.csv | cut -d, -f1-4
echo all_ok
