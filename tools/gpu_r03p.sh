#!/bin/bash
# round 3: 8-byte keyed partition records -- keyed parity (sort-free path suites), then the C4 leg
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03p
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py tests/test_gpu_exact.py -k "keyed" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03p/keyed.log 2>&1 || { grep -E "passed|failed|^FAILED|Error" gpurun_out/r03p/keyed.log | tail -5; exit 1; }
tail -1 gpurun_out/r03p/keyed.log
timeout -k 10 300 python3 -u tools/c4_ab.py 1 6 > gpurun_out/r03p/c4_compact.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/r03p/c4_compact.log; exit 1; }
SCOTTY_KG_NO_COMPACT=1 timeout -k 10 300 python3 -u tools/c4_ab.py 1 6 > gpurun_out/r03p/c4_12b.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/r03p/c4_12b.log; exit 1; }
echo compact; grep variant gpurun_out/r03p/c4_compact.log; echo 12B; grep variant gpurun_out/r03p/c4_12b.log
