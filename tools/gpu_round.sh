#!/bin/bash
# Full GPU pass: tests, smoke, bench, rocprof kernel stats.  Every GPU step has its own time limit; the
# script stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench_failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof_failed; exit 1; }
echo all_ok
