# keyed replay sort with a 4-bit last pass: keyed suites, then C4s default (4-bit last pass) vs c4s8 (8-bit) in one run
set -o pipefail
out=gpurun_out/r06/${1:-p26}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_keyed_sessions.py tests/test_gpu_keyed_count.py tests/test_gpu_keyed_lane_count.py tests/test_gpu_exact.py -m gpu -q --timeout 300 --timeout-method thread -k "keyed or Keyed or lane or session" > $out/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --skip-headline --no-cpu-baseline --only c4s,c4s8 > $out/c4s.json 2> $out/c4s.err || exit $?
python - <<PY
import json
d=json.load(open('$out/c4s.json'))['extra']
for k in ('c4s','c4s8'):
    r=d[k]['roofline']
    print(k, round(d[k]['value']/1e9,2), round(d[k]['ms_per_step'],3), {c: round(v*1e3,1) for c,v in r['device_ms_per_step_by_class'].items()})
PY
