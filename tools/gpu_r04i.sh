#!/bin/bash
# round 4: HBM traffic (separate --pmc passes) of the C4 keyed data pass and of the C2 ingest; C4 kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04i
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/r04i/pmc_kg_$c -o run --output-format csv -- python3 -u tools/c4_run.py 3 > gpurun_out/r04i/pmc_kg_$c.log 2>&1 || { echo pmc_kg_failed $c; tail -5 gpurun_out/r04i/pmc_kg_$c.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/r04i/pmc_ing_$c -o run --output-format csv -- python3 -u bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04i/pmc_ing_$c.log 2>&1 || { echo pmc_ing_failed $c; tail -5 gpurun_out/r04i/pmc_ing_$c.log; exit 1; }
done
python3 tools/keyed_traffic.py gpurun_out/r04i/pmc_kg_FETCH_SIZE gpurun_out/r04i/pmc_kg_WRITE_SIZE gpurun_out/r04i/keyed_traffic.json
python3 tools/ingest_traffic.py gpurun_out/r04i/pmc_ing_FETCH_SIZE gpurun_out/r04i/pmc_ing_WRITE_SIZE gpurun_out/r04i/ingest_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i/prof_c4 -o c4 --output-format csv -- python3 -u tools/c4_run.py 5 > gpurun_out/r04i/prof_c4.log 2>&1 || { echo prof_c4_failed; tail -5 gpurun_out/r04i/prof_c4.log; exit 1; }
f=$(find gpurun_out/r04i/prof_c4 -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | grep -v "at::" | head -16
