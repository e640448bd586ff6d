#!/bin/bash
# PMC passes over the C3 leg (exact batch path, 2^26 tuples per step): SQ stall / instruction-mix / LDS counters.
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/pmc_c3_$i -o run --output-format csv -- python -u bench.py --only c3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_c3_$i.log 2>&1 || { echo pmc_failed $i; tail -5 gpurun_out/pmc_c3_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_c3_1 gpurun_out/pmc_c3_2 > gpurun_out/pmc_c3_summary.txt
grep -E "xb_apply|xb_events|xb_tilemax|xb_classify" gpurun_out/pmc_c3_summary.txt
echo all_ok
