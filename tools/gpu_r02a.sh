#!/bin/bash
# Round-2 pass: GPU parity suite, smoke, C2 + C2s bench (no CPU baselines), rocprof kernel stats of that bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --only c2s > gpurun_out/bench_c2s.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench_c2s.log; exit 1; }
tail -1 gpurun_out/bench_c2s.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c2s > gpurun_out/prof_c2s.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c2s.log; exit 1; }
echo all_ok
