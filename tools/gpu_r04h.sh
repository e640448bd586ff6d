#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 400 python -u bench.py --only c2s --no-cpu-baseline --steps 5 > gpurun_out/r04h/bench.json 2> gpurun_out/r04h/bench.err || { echo bench_failed; tail -20 gpurun_out/r04h/bench.err; exit 1; }
grep "c2s:" gpurun_out/r04h/bench.err
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r04h/bench.json").read().strip().splitlines()[-1])
c = r["extra"]["c2s"]
print("c2s G/s %.1f ms %.4f frac %.3f" % (c["value"] / 1e9, c["ms_per_step"], c["roofline"]["frac"]),
      {k: round(v * 1e3, 1) for k, v in c["roofline"]["device_ms_per_step_by_class"].items()})
PY
timeout -k 10 300 python3 -u tools/ab_ingest.py --c2s --modes 6,7,6:1536,6:2048 --rounds 10 > gpurun_out/r04h/ab.json 2> gpurun_out/r04h/ab.err || { echo ab_failed; tail -5 gpurun_out/r04h/ab.err; exit 1; }
python3 -c "
import json
r = json.load(open('gpurun_out/r04h/ab.json'))
for k, v in r.items(): print(k, round(v['median_ms'] * 1e3, 1), 'us')
"
