#!/bin/bash
# PMC passes over the C4 leg (2^26 tuples per batch, sort-free keyed path): HBM bytes (FETCH_SIZE, WRITE_SIZE in
# passes of their own) and SQ occupancy / stall counters.  Summaries: tools/pmc_summary.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $pass -d gpurun_out/pmc_kg_$tag -o run --output-format csv -- python -u tools/c4_sweep.py 26 > gpurun_out/pmc_kg_$tag.log 2>&1 || { echo pmc_failed $tag; tail -5 gpurun_out/pmc_kg_$tag.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_kg_FETCH_SIZE gpurun_out/pmc_kg_WRITE_SIZE gpurun_out/pmc_kg_SQ_WAVES
echo all_ok
