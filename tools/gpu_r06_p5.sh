set -o pipefail
out=gpurun_out/r06/${1:-p5}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed_lane_count.py tests/test_gpu_keyed_count.py tests/test_gpu_exact.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python3 -u bench.py --skip-headline --no-cpu-baseline --only c4c > $out/c4c.json 2> $out/c4c.err || { echo "bench failed"; tail -5 $out/c4c.err; exit 1; }
echo bench done
