#!/bin/bash
# round 3: keyed scatter variants (persistent pipelined scatter 4, + bucket U=4 / U=8: 5 / 6) -- parity, then A/B
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03f
SCOTTY_TEST_KG_VARIANT=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_keyed_grid.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03f/keyed_grid_v4.log 2>&1 || { tail -40 gpurun_out/r03f/keyed_grid_v4.log; exit 1; }
tail -2 gpurun_out/r03f/keyed_grid_v4.log
timeout -k 10 500 python3 -u tools/c4_ab.py 1,4,5,6 6 > gpurun_out/r03f/c4_ab.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/r03f/c4_ab.log; exit 1; }
grep variant gpurun_out/r03f/c4_ab.log
