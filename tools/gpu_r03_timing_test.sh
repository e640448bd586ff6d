#!/bin/bash
# round 3: the timing-class test after the grid watermark's result-copy interval went away, then the grid suites
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03final/tests_parity_after_timing_fix.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03final/tests_parity_after_timing_fix.log | tail -6; exit 1; }
tail -1 gpurun_out/r03final/tests_parity_after_timing_fix.log
