#!/bin/bash
# C3 quiet path: kernel trace + stats of the C3 leg alone (20 steps incl. 2 pause steps)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/c3q
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c3q/prof -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/c3q/run.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/c3q/run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/c3q/prof/run_kernel_trace.csv > gpurun_out/c3q/steps.txt
cat gpurun_out/c3q/steps.txt
tail -1 gpurun_out/c3q/run.log | cut -c1-600
