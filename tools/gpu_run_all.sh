#!/bin/bash
# usage: run_all.sh [tests] [bench] [prof]
export TMPDIR=/tmp
for what in "$@"; do
  case $what in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$? >> gpurun_out/gpu_tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke_rc=$? >> gpurun_out/smoke.log ;;
    bench) timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; echo bench_rc=$? >> gpurun_out/bench.log ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; echo prof_rc=$? >> gpurun_out/prof.log ;;
  esac
done
