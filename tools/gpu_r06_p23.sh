# count path: four range searches in parallel lanes, the window aggregation's count-measure searches by lane groups
set -o pipefail
out=gpurun_out/r06/${1:-p23}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_count.py tests/test_golden.py tests/test_gpu_shard.py tests/test_gpu_poison.py tests/test_gpu_exact.py -m gpu -q --timeout 300 --timeout-method thread -k "count or Count or golden or shard or poison" > $out/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --skip-headline --only c5,c5t --no-cpu-baseline > $out/c5.json 2> $out/c5.err || exit $?
python - <<PY
import json
d=json.load(open('$out/c5.json'))['extra']
for k in ('c5','c5t'):
    r=d[k]['roofline']
    print(k, round(d[k]['value']/1e9,1), round(d[k]['ms_per_step'],4), {c: round(v*1e3,1) for c,v in r['device_ms_per_step_by_class'].items()})
PY
