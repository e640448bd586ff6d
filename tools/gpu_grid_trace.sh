#!/bin/bash
# Grid path parity + C2/C2s bench (tools/gpu_grid.sh), then a kernel + copy trace of the headline with the per-step
# kernel sequence and the gaps between launches (tools/step_gaps.py).
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_grid.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_c2gap -o run --output-format csv -- python -u bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/prof_c2gap.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c2gap.log; exit 1; }
python3 tools/step_gaps.py gpurun_out/prof_c2gap ingest_kernel 12 18
echo all_ok
