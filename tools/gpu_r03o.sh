#!/bin/bash
# round 3: C4 keyed leg counters -- SQ issue/LDS counters, and HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03o
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/r03o/pmc_sq -o run --output-format csv -- python3 -u tools/leg_run.py c4 > gpurun_out/r03o/pmc_sq.log 2>&1 || { echo pmc_failed sq; tail -5 gpurun_out/r03o/pmc_sq.log; exit 1; }
echo sq_done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/r03o/pmc_$c -o run --output-format csv -- python3 -u tools/leg_run.py c4 > gpurun_out/r03o/pmc_$c.log 2>&1 || { echo pmc_failed $c; tail -5 gpurun_out/r03o/pmc_$c.log; exit 1; }
  echo ${c}_done
done
python3 tools/pmc_summary.py gpurun_out/r03o/pmc_sq > gpurun_out/r03o/c4_sq.txt
python3 tools/pmc_summary.py gpurun_out/r03o/pmc_FETCH_SIZE gpurun_out/r03o/pmc_WRITE_SIZE > gpurun_out/r03o/c4_traffic.txt
grep -E "kg_|lane_|scan" gpurun_out/r03o/c4_sq.txt | cut -c1-250
grep -E "kg_|lane_|scan" gpurun_out/r03o/c4_traffic.txt | cut -c1-200
