#!/bin/bash
# C3 exact batch path: non-keyed exact-engine parity tests, then the C3 leg under a kernel trace (per-step breakdown).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_golden.py -k "not keyed" -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/c3_tests.log; exit 1; }
tail -2 gpurun_out/c3_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c3 -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c3 --steps 3 --warmup 1 > gpurun_out/prof_c3.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c3.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/prof_c3/run_kernel_trace.csv | tee gpurun_out/c3_steps.txt
python3 -c "import json; r=json.loads(open('gpurun_out/prof_c3.log').read().strip().splitlines()[-1]); c=r['extra']['c3']; print('C3', c['value']/1e9, 'G t/s', c['ms_per_step'], 'ms/step (under trace)')"
echo c3_ok
