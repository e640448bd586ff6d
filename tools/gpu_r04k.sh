#!/bin/bash
# round 4: validation of the start band (SCOTTY_QUIET_BAND=1: every exact operator uses it) and of keyed scatter
# variant 2, then same-box A/B: C3 with / without the band, C4 variant 1 / 2
set -o pipefail
mkdir -p gpurun_out/r04k
export SCOTTY_QUIET_BAND=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_poison.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04k/tests_band_exact.log 2>&1 || { echo band_exact_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04k/tests_band_exact.log | tail -15; exit 1; }
grep -E "windows [0-9]+, band|passed|failed" gpurun_out/r04k/tests_band_exact.log | tail -12
timeout -k 10 240 python -u bench.py --no-cpu-baseline --only c3 --steps 3 --warmup 1 > gpurun_out/r04k/bench_c3_band.json 2> gpurun_out/r04k/bench_c3_band.err || { echo bench_c3_band_failed; tail -5 gpurun_out/r04k/bench_c3_band.err; exit 1; }
SCOTTY_QUIET_BAND=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --only c3 --steps 3 --warmup 1 > gpurun_out/r04k/bench_c3_noband.json 2> gpurun_out/r04k/bench_c3_noband.err || { echo bench_c3_noband_failed; tail -5 gpurun_out/r04k/bench_c3_noband.err; exit 1; }
python3 - <<'PY'
import json
for f in ("band", "noband"):
    d = json.loads(open("gpurun_out/r04k/bench_c3_%s.json" % f).read().strip().splitlines()[-1])
    e = d["extra"]["c3"]
    print(f, round(e["value"] / 1e9, 1), "G/s", round(e["ms_per_step"], 3), "ms", e["ms_per_step_each"], "moves", e.get("start_band_moves"), "pieces", e.get("jump_pieces"), "rounds", e["events_rounds_each"])
PY
SCOTTY_TEST_KG_VARIANT=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_grid.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r04k/tests_keyed_v2.log 2>&1 || { echo keyed_v2_tests_failed; grep -E "passed|failed|Error|assert" gpurun_out/r04k/tests_keyed_v2.log | tail -15; exit 1; }
tail -1 gpurun_out/r04k/tests_keyed_v2.log
timeout -k 10 400 python -u tools/ab_c4.py 1 2 > gpurun_out/r04k/ab_c4.json 2> gpurun_out/r04k/ab_c4.err || { echo ab_c4_failed; tail -5 gpurun_out/r04k/ab_c4.err; exit 1; }
cat gpurun_out/r04k/ab_c4.json
