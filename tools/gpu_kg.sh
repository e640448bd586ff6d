#!/bin/bash
# Keyed engine: parity (sort-free path tests + keyed exact-engine tests), then the C4 leg and its kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py tests/test_gpu_exact.py -k "keyed or kg or grid" -x -q --timeout 300 --timeout-method thread > gpurun_out/kg_tests.log 2>&1 || { echo kg_tests_failed; tail -40 gpurun_out/kg_tests.log; exit 1; }
tail -2 gpurun_out/kg_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c4 > gpurun_out/prof_c4.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c4.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('gpurun_out/prof_c4.log') if l.startswith('{')][-1]); c=r['extra']['c4']; print('C4 (under trace)', c['value']/1e9, 'G t/s', c['ms_per_step'], 'ms/step')"
python3 tools/trace_steps.py gpurun_out/prof_c4/run_kernel_trace.csv --first kg_prep_kernel --steps 3 --median | tee gpurun_out/c4_steps.txt
echo all_ok
