#!/bin/bash
# round 6: full -m gpu suite + the bench legs touched this round (C1 warm-up, C5/C5t device classes, C4 host rows,
# PCIe placement, kernel names); $1 = tag
set -o pipefail
tag=${1:-r06a}
out=gpurun_out/r06/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|Error" $out/gpu_tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --skip-headline --no-cpu-baseline --only c1,c5,c5t,c4,pcie > $out/bench_legs.json 2> $out/bench_legs.err
