#!/bin/bash
# Round-1 re-check: GPU parity suite, smoke, C4 batch sweep.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; exit 1; }
timeout -k 10 400 python -u tools/c4_sweep.py 24 25 26 > gpurun_out/c4_sweep.log 2>&1 || { echo c4_failed; tail -20 gpurun_out/c4_sweep.log; exit 1; }
cat gpurun_out/c4_sweep.log
echo all_ok
