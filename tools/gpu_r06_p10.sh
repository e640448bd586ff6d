set -o pipefail
out=gpurun_out/r06/${1:-p10}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_band.py tests/test_golden.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_count.py tests/test_gpu_poison.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for t in none exact_wm_fused=0; do
    tune=""; [ $t != none ] && tune="--tune $t"
    timeout -k 10 300 python3 -u bench.py --skip-headline --no-cpu-baseline --only c3 $tune > $out/ab_c3_${t}_$r.json 2> $out/ab_c3_${t}_$r.err || { echo "c3 A/B $t failed"; exit 1; }
  done
done
echo "c3 A/B done"
timeout -k 10 400 python3 -u bench.py --skip-headline --no-cpu-baseline --only c5,c5t > $out/c5.json 2> $out/c5.err || { echo "bench failed"; exit 1; }
echo "c5 done"
