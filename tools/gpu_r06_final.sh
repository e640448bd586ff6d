#!/bin/bash
# Round-6 final pass on the current tree: the full -m gpu suite, smoke(), the default bench line.  Each step under its
# own time limit; the chain stops at the first failure.
set -o pipefail
out=gpurun_out/r06/${1:-final}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests_full.txt 2>&1 \
  || { echo "suite failed"; tail -40 $out/gpu_tests_full.txt; exit 1; }
tail -1 $out/gpu_tests_full.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.txt; exit 1; }
tail -2 $out/smoke.txt
timeout -k 10 600 python3 -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -10 $out/bench.err; exit 1; }
echo "bench done"
# the sharded C2 at N=1 (RCCL exchange on the op's stream vs host-synchronised), 100 steps each, alternated
if [ -n "$SHARD_AB" ]; then
  for mode in sync async; do
    if [ $mode = sync ]; then export SCOTTY_SHARD_SYNC=1; else export SCOTTY_SHARD_SYNC=0; fi
    timeout -k 10 300 python -u bench.py --shard --no-extra --no-cpu-baseline --steps 100 > $out/c2_shard_$mode.json 2> $out/c2_shard_$mode.err || exit $?
    python -c "import json; d=json.load(open('$out/c2_shard_$mode.json')); print('$mode', round(d['value']/1e9,1), round(d['ms_per_step'],4))"
  done
fi
