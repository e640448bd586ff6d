#!/bin/bash
# PMC passes over the C3 leg (exact batch path, 2^26 tuples per step): HBM bytes and SQ stall / LDS counters.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in "FETCH_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $pass -d gpurun_out/pmc_c3_$tag -o run --output-format csv -- python -u bench.py --only c3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_c3_$tag.log 2>&1 || { echo pmc_failed $tag; tail -5 gpurun_out/pmc_c3_$tag.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_c3_FETCH_SIZE gpurun_out/pmc_c3_SQ_WAVES > gpurun_out/pmc_c3_summary.txt
echo all_ok
