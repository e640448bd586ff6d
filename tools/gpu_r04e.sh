#!/bin/bash
# round 4: C2 per-kernel profile (commit / wm_prep / wm_windows / cix_build) + the achievable read rate
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04e
timeout -k 10 120 ./tools/read_roof > gpurun_out/r04e/read_roof.txt 2>&1 || { echo roof_failed; cat gpurun_out/r04e/read_roof.txt; exit 1; }
cat gpurun_out/r04e/read_roof.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04e/prof -o c2 --output-format csv -- python3 -u bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/r04e/bench.json 2> gpurun_out/r04e/bench.err || { echo prof_failed; tail -20 gpurun_out/r04e/bench.err; exit 1; }
f=$(find gpurun_out/r04e/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -14
