#!/bin/bash
# round 3: kernel breakdown of C3's pause step with a 16k-tuple event-exact prefix
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03u
SCOTTY_XQ_CHUNK=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03u/c3prof -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/r03u/c3_run.log 2>&1 || { echo c3_prof_failed; tail -20 gpurun_out/r03u/c3_run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/r03u/c3prof/run_kernel_trace.csv > gpurun_out/r03u/c3_steps.txt
python3 tools/trace_c3.py --marker xb_prep_kernel gpurun_out/r03u/c3prof/run_kernel_trace.csv > gpurun_out/r03u/c3_rounds.txt
cat gpurun_out/r03u/c3_steps.txt gpurun_out/r03u/c3_rounds.txt
