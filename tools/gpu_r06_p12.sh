# count-path check after the first-walk copy-source fix: the small-pushes tests under two poison values, then the
# count/shard/golden/poison suites; stops at the first abort, fault or time limit
set -o pipefail
out=gpurun_out/r06/${1:-p12}
mkdir -p $out
stop() { case $1 in 124|134|137|139) echo "stopping after rc=$1"; exit $1;; esac; }
for p in none 0xA5; do
  if [ $p = none ]; then unset SCOTTY_ALLOC_POISON; else export SCOTTY_ALLOC_POISON=$p; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_count.py -m gpu -q --timeout 120 --timeout-method thread \
    -k "small_pushes or time_windows_on_count_path" > $out/count_$p.log 2>&1; rc=$?; echo "poison $p rc=$rc"
  tail -2 $out/count_$p.log; stop $rc
done
unset SCOTTY_ALLOC_POISON
timeout -k 10 600 python -u -m pytest tests/test_gpu_count.py tests/test_gpu_shard.py tests/test_golden.py \
  tests/test_gpu_poison.py -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $out/tests.log
