set -o pipefail
out=gpurun_out/r06/${1:-p11}
mkdir -p $out
for p in none 0xA5 0x00 0xFF; do
  if [ $p = none ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_count.py -m gpu -q --timeout 120 --timeout-method thread -k "small_pushes or time_windows_on_count_path" > $out/count_$p.log 2>&1; echo "poison $p rc=$?"
  else
    SCOTTY_ALLOC_POISON=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_count.py -m gpu -q --timeout 120 --timeout-method thread -k "small_pushes or time_windows_on_count_path" > $out/count_$p.log 2>&1; echo "poison $p rc=$?"
  fi
  tail -2 $out/count_$p.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_count.py tests/test_gpu_shard.py tests/test_golden.py tests/test_gpu_poison.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; echo "suite rc=$?"; tail -2 $out/tests.log
