#!/bin/bash
# SQ counters of the C4 data-pass kernels (what bounds kg_scatter / kg_bucket / kg_hist): two passes of <= 8 SQ
# counters each, separate runs, per-dispatch values kept compressed.  $1 = tag
set -o pipefail
out=gpurun_out/r06/${1:-c4sq}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
a="--skip-headline --no-cpu-baseline --only c4"
p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
p2="SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -k 10 500 rocprofv3 --output-format csv --pmc $p -d $out/sq$i -o run -- python3 -u bench.py $a > $out/sq$i.json 2> $out/sq$i.err \
    || { echo "pass $i failed"; exit 1; }
  find $out/sq$i -type f ! -name "*counter_collection.csv" -size +256k -delete
  find $out/sq$i -type f -name "*.csv" -size +64k -exec gzip -9 {} \;
  echo "pass $i done"
done
python3 tools/sq_summary.py $out > $out/summary.txt 2>&1 || true
