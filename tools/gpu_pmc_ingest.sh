#!/bin/bash
# HBM traffic of the C2 ingest kernel on the committed code: FETCH_SIZE and WRITE_SIZE in separate --pmc passes.
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_ing_$c -o run --output-format csv -- python -u bench.py --no-extra --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_ing_$c.log 2>&1 || { echo pmc_failed $c; tail -5 gpurun_out/pmc_ing_$c.log; exit 1; }
done
python3 tools/ingest_traffic.py gpurun_out/pmc_ing_FETCH_SIZE gpurun_out/pmc_ing_WRITE_SIZE gpurun_out/ingest_traffic.json
echo all_ok
