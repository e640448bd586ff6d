#!/bin/bash
# round 4: ingest variants on the C2 and C2s streams (interleaved rounds, HIP-event ingest time per push)
set -o pipefail
mkdir -p gpurun_out/r04f
for w in c2 c2s; do
  extra=""; [ $w = c2s ] && extra="--c2s"
  timeout -k 10 300 python3 -u tools/ab_ingest.py $extra --modes 6,6:768,7:256,7:384,7:448,7:512,7:576,7:640 --rounds 16 > gpurun_out/r04f/ab_$w.json 2> gpurun_out/r04f/ab_$w.err || { echo ab_failed; tail -20 gpurun_out/r04f/ab_$w.err; exit 1; }
  echo "== $w"
  python3 -c "
import json
r = json.load(open('gpurun_out/r04f/ab_$w.json'))
for k, v in r.items(): print(k, round(v['median_ms'] * 1e3, 1), 'us', round(v['median_TBps'], 3), 'TB/s')
"
done
