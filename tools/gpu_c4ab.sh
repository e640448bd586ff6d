#!/bin/bash
# C4 A/B of the sort-free path's kernel variants + a kernel trace of each.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/c4ab.log
for v in 1 3; do
  timeout -k 10 300 python -u tools/c4_sweep.py 26 keyed_grid_variant=$v >> gpurun_out/c4ab.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/c4ab.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c4v$v -o run --output-format csv -- python -u tools/c4_sweep.py 26 keyed_grid_variant=$v > gpurun_out/prof_c4v$v.log 2>&1 || { echo prof_failed; exit 1; }
  python3 tools/trace_steps.py gpurun_out/prof_c4v$v/run_kernel_trace.csv --first kg_prep_kernel --steps 3 --median | head -6
done
grep '^{' gpurun_out/c4ab.log | python3 -c "import sys,json; [print(r['tune'], round(r['value']/1e9,2), 'G t/s', round(r['ms_per_step'],3), 'ms') for r in map(json.loads, sys.stdin)]"
echo all_ok
