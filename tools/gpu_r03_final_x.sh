#!/bin/bash
# round-3 evidence after the last engine changes: the exact suite (event-exact round control via one copy launch and
# a device-side resume fill), then part B (bench line + C2 ingest PMC traffic) and part C (per-leg rocprofv3 runs)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03final/tests_exact.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03final/tests_exact.log | tail -6; exit 1; }
tail -1 gpurun_out/r03final/tests_exact.log
bash tools/gpu_r03_final_b.sh && bash tools/gpu_r03_final_c.sh
