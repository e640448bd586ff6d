#!/bin/bash
# round 3: smoke on the final tree
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03final/smoke_final_tree.log 2>&1 || { echo smoke_failed; tail -5 gpurun_out/r03final/smoke_final_tree.log; exit 1; }
tail -1 gpurun_out/r03final/smoke_final_tree.log
