#!/bin/bash
# Keyed-path check: keyed GPU parity tests, then the C4 batch sweep and its kernel stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_shard.py -m gpu -q -x -k "keyed or shard" --timeout 200 --timeout-method thread > gpurun_out/keyed_tests.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/keyed_tests.log; exit 1; }
tail -2 gpurun_out/keyed_tests.log
timeout -k 10 300 python -u tools/c4_sweep.py 24 26 > gpurun_out/c4_sweep.log 2>&1 || { echo c4_failed; tail -20 gpurun_out/c4_sweep.log; exit 1; }
cat gpurun_out/c4_sweep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python -u tools/c4_sweep.py 26 > gpurun_out/prof_c4.log 2>&1 || { echo prof_failed; exit 1; }
echo all_ok
