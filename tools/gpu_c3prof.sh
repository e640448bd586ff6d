#!/bin/bash
# C3 (exact batch path) kernel trace: per-step breakdown of the exact engine's batch-parallel passes.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c3 -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c3 --steps 3 --warmup 1 > gpurun_out/prof_c3.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c3.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/prof_c3/run_kernel_trace.csv
echo c3_ok
