#!/bin/bash
# Full GPU pass: tests, smoke, bench, rocprof kernel stats.  Every GPU step has its own time limit; the
# script stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests_failed; grep -E "^FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench_failed; tail -5 gpurun_out/bench.log; exit 1; }
echo bench_ok
echo all_ok
