#!/bin/bash
# Smoke, the full bench line (all legs + CPU baselines) and a rocprofv3 kernel-stats pass of the same bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_bench.log; exit 1; }
head -24 gpurun_out/prof_bench/run_kernel_stats.csv | cut -d, -f1-4
echo all_ok
