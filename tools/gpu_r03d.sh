#!/bin/bash
# round 3: keyed parity after the key-interleaved store, then kernel traces of the C3 and C4 legs
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03d
timeout -k 10 500 python -u -m pytest tests/test_gpu_keyed_grid.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03d/keyed_grid.log 2>&1 || { tail -40 gpurun_out/r03d/keyed_grid.log; exit 1; }
tail -2 gpurun_out/r03d/keyed_grid.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03d/c3 -o run --output-format csv -- python3 -u tools/c3_run.py 10 > gpurun_out/r03d/c3_run.log 2>&1 || { echo c3_prof_failed; tail -20 gpurun_out/r03d/c3_run.log; exit 1; }
python3 tools/trace_c3.py gpurun_out/r03d/c3/run_kernel_trace.csv > gpurun_out/r03d/c3_steps.txt
python3 tools/trace_c3.py --marker xb_prep gpurun_out/r03d/c3/run_kernel_trace.csv > gpurun_out/r03d/c3_pause_rounds.txt
cat gpurun_out/r03d/c3_steps.txt
head -30 gpurun_out/r03d/c3_pause_rounds.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03d/c4 -o run --output-format csv -- python3 -u tools/c4_run.py 6 > gpurun_out/r03d/c4_run.log 2>&1 || { echo c4_prof_failed; tail -20 gpurun_out/r03d/c4_run.log; exit 1; }
python3 tools/trace_c4.py gpurun_out/r03d/c4/run_kernel_trace.csv > gpurun_out/r03d/c4_steps.txt
cat gpurun_out/r03d/c4_steps.txt
tail -1 gpurun_out/r03d/c4_run.log | cut -c1-1500
