#!/bin/bash
# Full bench line (with CPU baseline) and a rocprofv3 kernel-stats pass of the same bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_bench.log; exit 1; }
echo all_ok
