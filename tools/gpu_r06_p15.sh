# RCCL exchange on the op's own stream (ExternalStream) vs host-synchronised: the 1-rank RCCL parity tests, then
# the sharded C2 at N=1 alternated between the two modes (100 timed steps each)
set -o pipefail
out=gpurun_out/r06/${1:-p15}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -v --timeout 240 --timeout-method thread \
  -k rccl > $out/shard_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $out/shard_tests.txt; [ $rc -eq 0 ] || exit $rc
for mode in sync async sync async; do
  if [ $mode = sync ]; then export SCOTTY_SHARD_SYNC=1; else export SCOTTY_SHARD_SYNC=0; fi
  timeout -k 10 300 python -u bench.py --shard --no-extra --no-cpu-baseline --steps 100 > $out/tmp.json 2> $out/c2_shard_$mode.err || exit $?
  cat $out/tmp.json >> $out/c2_shard_$mode.jsonl
  python -c "import json,sys; d=json.load(open('$out/tmp.json')); print('$mode', round(d['value']/1e9,1), round(d['ms_per_step'],4), d['config']['parallelism'][-30:])"
done
rm $out/tmp.json
