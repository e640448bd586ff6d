#!/bin/bash
# round 4: the exact engine's start band -- band / full-size / exact parity suites, then the C3 bench leg
set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 800 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread -k "band or c3" > gpurun_out/r04j/tests_band.log 2>&1 || { echo band_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04j/tests_band.log | tail -15; exit 1; }
grep -E "passed|failed" gpurun_out/r04j/tests_band.log | tail -3
timeout -k 10 300 python -u bench.py --no-cpu-baseline --only c3 --steps 20 --warmup 3 > gpurun_out/r04j/bench_c3.json 2> gpurun_out/r04j/bench_c3.err || { echo bench_failed; tail -5 gpurun_out/r04j/bench_c3.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r04j/bench_c3.json').read().strip().splitlines()[-1])
for l in d.get('extra',[]):
  print({k:l.get(k) for k in ('config','value','ms_per_step','step_ms','pause_step_ms')}) if isinstance(l,dict) else None
print(json.dumps(d.get('extra'))[:1500])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r04j/tests_exact.log 2>&1 || { echo exact_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04j/tests_exact.log | tail -15; exit 1; }
tail -2 gpurun_out/r04j/tests_exact.log
timeout -k 10 400 python -u tools/ab_c4.py 1 2 > gpurun_out/r04j/ab_c4.json 2> gpurun_out/r04j/ab_c4.err || { echo ab_c4_failed; tail -5 gpurun_out/r04j/ab_c4.err; exit 1; }
cat gpurun_out/r04j/ab_c4.json
SCOTTY_TEST_KG_VARIANT=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r04j/tests_keyed.log 2>&1 || { echo keyed_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04j/tests_keyed.log | tail -15; exit 1; }
tail -2 gpurun_out/r04j/tests_keyed.log
timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline > gpurun_out/r04j/bench_c2.json 2> gpurun_out/r04j/bench_c2.err || { echo bench_c2_failed; tail -5 gpurun_out/r04j/bench_c2.err; exit 1; }
tail -1 gpurun_out/r04j/bench_c2.json | cut -c1-600
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread -k "not c3" > gpurun_out/r04j/tests_grid.log 2>&1 || { echo grid_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04j/tests_grid.log | tail -15; exit 1; }
tail -2 gpurun_out/r04j/tests_grid.log
