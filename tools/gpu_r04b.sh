#!/bin/bash
# round 4: C3 full-size + the prefix split, with the quiet-attempt trace
set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "c3" -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r04b/c3.log 2>&1 || { echo c3_failed; grep -E "attempts|PASS|FAIL|Error" gpurun_out/r04b/c3.log | tail -40; exit 1; }
grep -E "attempts|commits|PASS|FAIL" gpurun_out/r04b/c3.log | tail -40
