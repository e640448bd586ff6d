#!/bin/bash
# Exact-engine / count-path parity (LazySlice record sets), then the grid-path A/B + profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_count.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_exact.log 2>&1 || { echo tests_failed; tail -60 gpurun_out/gpu_exact.log; exit 1; }
tail -3 gpurun_out/gpu_exact.log
bash tools/gpu_r02b.sh
