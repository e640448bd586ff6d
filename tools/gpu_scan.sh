#!/bin/bash
# int32 scan check (tools/scan_check, built in-tree: hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include -o
# tools/scan_check tools/scan_check.hip), keyed + exact-engine parity, then C3 / C4 bench legs and the C4 trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/scan_check > gpurun_out/scan_check.log 2>&1 || { echo scan_check_failed; tail -20 gpurun_out/scan_check.log; exit 1; }
tail -1 gpurun_out/scan_check.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_keyed_grid.py tests/test_gpu_exact.py tests/test_gpu_count.py -x -q --timeout 300 --timeout-method thread > gpurun_out/scan_tests.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/scan_tests.log; exit 1; }
tail -1 gpurun_out/scan_tests.log
timeout -k 10 400 python -u bench.py --only c3,c4 --no-cpu-baseline > gpurun_out/bench_scan.log 2>&1 || { echo bench_failed; tail -5 gpurun_out/bench_scan.log; exit 1; }
python3 -c "
import json; r=json.loads([l for l in open('gpurun_out/bench_scan.log') if l.startswith('{')][-1])
[print(k, round(r['extra'][k]['value']/1e9,2), 'G t/s', round(r['extra'][k]['ms_per_step'],3), 'ms') for k in ('c3','c4')]"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_c4s -o run --output-format csv -- python -u tools/c4_sweep.py 26 > gpurun_out/prof_c4s.log 2>&1 || { echo prof_failed; exit 1; }
python3 tools/step_gaps.py gpurun_out/prof_c4s kg_prep_kernel 62 63
echo all_ok
