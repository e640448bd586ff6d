set -o pipefail
out=gpurun_out/r06/${1:-p7}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py tests/test_gpu_first.py tests/test_gpu_band.py tests/test_gpu_f64_signed.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --only c1,c2s,c3 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
echo bench done
