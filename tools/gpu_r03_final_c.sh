#!/bin/bash
# round-3 evidence, part C: every bench leg in its own rocprofv3 kernel-trace + stats run (C2 = bench.py --no-extra)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03final/prof_c2 -o run --output-format csv -- python3 -u bench.py --no-extra --no-cpu-baseline > gpurun_out/r03final/prof_c2.log 2>&1 || { echo prof_failed c2; tail -5 gpurun_out/r03final/prof_c2.log; exit 1; }
echo prof_c2_ok
for leg in c1 c2s c3 c4 c5 c5t; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03final/prof_$leg -o run --output-format csv -- python3 -u tools/leg_run.py $leg > gpurun_out/r03final/prof_$leg.log 2>&1 || { echo prof_failed $leg; tail -5 gpurun_out/r03final/prof_$leg.log; exit 1; }
  echo prof_${leg}_ok
done
python3 tools/leg_stats.py gpurun_out/r03final > gpurun_out/r03final/leg_kernel_stats.txt
grep -E "^==|dominant" gpurun_out/r03final/leg_kernel_stats.txt
