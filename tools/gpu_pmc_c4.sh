#!/bin/bash
# One PMC pass (SQ issue/stall counters) over the C4 leg at 2^24 tuples per batch.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM -d gpurun_out/pmc_c4 -o run --output-format csv -- python -u tools/c4_sweep.py 24 > gpurun_out/pmc_c4.log 2>&1 || { echo pmc_failed; tail -5 gpurun_out/pmc_c4.log; exit 1; }
echo all_ok
