# sharded C2 at N=1: host-synchronised vs device-event exchange, alternated, 100 timed steps (inputs of every step resident: 200 do not fit) each
set -o pipefail
out=gpurun_out/r06/${1:-p14}
mkdir -p $out
for mode in sync async sync async; do
  if [ $mode = sync ]; then export SCOTTY_SHARD_SYNC=1; else export SCOTTY_SHARD_SYNC=0; fi
  timeout -k 10 300 python -u bench.py --shard --no-extra --no-cpu-baseline --steps 100 > $out/tmp.json 2> $out/c2_shard_$mode.err || exit $?
  cat $out/tmp.json >> $out/c2_shard_$mode.jsonl
  python -c "import json,sys; d=json.load(open('$out/tmp.json')); print('$mode', round(d['value']/1e9,1), round(d['ms_per_step'],4), d['config']['parallelism'][-30:])"
done
rm $out/tmp.json
