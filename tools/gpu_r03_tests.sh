#!/bin/bash
# round-3 evidence, part A: the full -m gpu suite and the smoke test on the committed tree
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03final/gpu_tests.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r03final/gpu_tests.log | tail -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03final/smoke.log 2>&1 || { echo smoke_failed; tail -5 gpurun_out/r03final/smoke.log; exit 1; }
tail -1 gpurun_out/r03final/smoke.log
