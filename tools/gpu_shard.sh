#!/bin/bash
# Sharded (time-range) path: 2-rank GPU parity (gloo) and the N=1 RCCL rehearsal of the bench's sharded C2 under a
# kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { echo shard_tests_failed; tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -1 gpurun_out/shard_tests.log
timeout -k 10 200 python -u bench.py --shard --no-extra --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_shard1.log 2>&1 || { echo bench_failed; tail -5 gpurun_out/bench_shard1.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('gpurun_out/bench_shard1.log') if l.startswith('{')][-1]); print('shard N=1', r['value']/1e9, 'G/s', r['ms_per_step'], 'ms/step')"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_shard -o run --output-format csv -- python -u bench.py --shard --no-extra --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_shard.log 2>&1 || { echo prof_failed; exit 1; }
echo all_ok
