#!/bin/bash
# The full -m gpu suite, once; $1 = tag (output dir gpurun_out/$1), $2 = allocation poison byte or "off"
set -o pipefail
tag=${1:-suite}; poison=${2:-off}
mkdir -p gpurun_out/$tag
if [ "$poison" != off ]; then export SCOTTY_ALLOC_POISON=$poison; fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|Error" gpurun_out/$tag/gpu_tests.log | tail -8
exit $rc
