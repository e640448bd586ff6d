# RCCL exchange ordered by device events vs host-synchronised: the 1-rank RCCL parity tests, then the sharded C2
# headline at N=1 in both modes beside the unsharded one (and the C5 legs sharded, both modes)
set -o pipefail
out=gpurun_out/r06/${1:-p13}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -v --timeout 240 --timeout-method thread \
  -k rccl > $out/shard_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $out/shard_tests.txt; [ $rc -eq 0 ] || exit $rc
for mode in async sync; do
  if [ $mode = sync ]; then export SCOTTY_SHARD_SYNC=1; else export SCOTTY_SHARD_SYNC=0; fi
  timeout -k 10 300 python -u bench.py --shard --no-extra --no-cpu-baseline --steps 40 > $out/c2_shard_$mode.json 2> $out/c2_shard_$mode.err || exit $?
  echo "$mode: $(head -c 400 $out/c2_shard_$mode.json)"
done
timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --steps 40 > $out/c2_plain.json 2> $out/c2_plain.err || exit $?
echo "plain: $(head -c 300 $out/c2_plain.json)"
