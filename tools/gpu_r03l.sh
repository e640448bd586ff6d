#!/bin/bash
# round 3: why the C3 ingest is slower than C2s': one SQ counter pass over each leg, plus the mode-7 (pipelined) A/B
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03l
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for leg in c3 c2s; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/r03l/pmc_$leg -o run --output-format csv -- python3 -u tools/leg_run.py $leg > gpurun_out/r03l/pmc_$leg.log 2>&1 || { echo pmc_failed $leg; tail -5 gpurun_out/r03l/pmc_$leg.log; exit 1; }
  echo "pmc $leg done"
  python3 tools/pmc_summary.py gpurun_out/r03l/pmc_$leg | grep -i "ingest" | head -4
done
SCOTTY_INGEST_MODE=7 timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03l/c3_mode7.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/r03l/c3_mode7.log; exit 1; }
grep '^{' gpurun_out/r03l/c3_mode7.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('mode7', round(d['ms_per_step'],4), 'ingest_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3))"
