set -o pipefail
out=gpurun_out/r06/${1:-p8}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_count.py tests/test_golden.py tests/test_gpu_shard.py tests/test_gpu_poison.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python3 -u bench.py --skip-headline --no-cpu-baseline --only c5,c5t > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
echo bench done
