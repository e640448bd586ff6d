#!/bin/bash
# round-3 evidence, part B: the bench line (default command) and the C2 ingest HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate passes); part C (tools/gpu_r03_final_c.sh) profiles every leg in its own rocprofv3 run
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03final
timeout -k 10 600 python -u bench.py > gpurun_out/r03final/bench.json 2> gpurun_out/r03final/bench.log || { echo bench_failed; tail -5 gpurun_out/r03final/bench.log; exit 1; }
echo bench_ok
python3 -c "
import json; d=json.load(open('gpurun_out/r03final/bench.json'))
print('C2', round(d['value']/1e9,1), 'ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'frac_step', round(d['roofline']['frac_step'],3))
for k,x in d.get('extra',{}).items():
    r=x.get('roofline') or {}
    print(k, round(x.get('value',0)/1e9,2), 'ms', round(x.get('ms_per_step',0),4), 'frac', round(r.get('frac',0),3), 'cpu', round((x.get('cpu_baseline') or {}).get('value',0)/1e6,1))
"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/r03final/pmc_ing_$c -o run --output-format csv -- python3 -u bench.py --no-extra --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03final/pmc_ing_$c.log 2>&1 || { echo pmc_failed $c; tail -5 gpurun_out/r03final/pmc_ing_$c.log; exit 1; }
done
python3 tools/ingest_traffic.py gpurun_out/r03final/pmc_ing_FETCH_SIZE gpurun_out/r03final/pmc_ing_WRITE_SIZE gpurun_out/r03final/ingest_traffic.json
cat gpurun_out/r03final/ingest_traffic.json | head -c 600
