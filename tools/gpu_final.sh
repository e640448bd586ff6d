#!/bin/bash
# Round-end evidence: full -m gpu suite, smoke, the bench line, and a rocprofv3 kernel-stats/trace pass of the bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests_failed; grep -E "^FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench_failed; tail -5 gpurun_out/bench.log; exit 1; }
echo bench_ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_final.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_final.log; exit 1; }
echo all_ok
