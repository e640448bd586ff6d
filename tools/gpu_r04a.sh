#!/bin/bash
# round 4: poisoned-allocation regression + oracle parity at bench sizes
set -o pipefail
mkdir -p gpurun_out/r04a
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_poison.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/poison.log 2>&1 || { echo poison_failed; tail -40 gpurun_out/r04a/poison.log; exit 1; }
tail -3 gpurun_out/r04a/poison.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py "tests/test_gpu_exact.py::test_config3_full_size_quiet_path_equals_replay" -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r04a/full.log 2>&1 || { echo full_failed; tail -40 gpurun_out/r04a/full.log; exit 1; }
tail -3 gpurun_out/r04a/full.log
