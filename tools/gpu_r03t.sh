#!/bin/bash
# round 3: A/B of the event-exact prefix a batch starting with a session-gap jump gets (SCOTTY_XQ_CHUNK tuples)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r03t
for c in 16384 65536 262144 1048576; do
  SCOTTY_XQ_CHUNK=$c timeout -k 10 300 python3 -u tools/c3_run.py 10 > gpurun_out/r03t/c3_chunk$c.log 2>&1 || { echo c3_failed $c; tail -20 gpurun_out/r03t/c3_chunk$c.log; exit 1; }
  grep '^{' gpurun_out/r03t/c3_chunk$c.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d["roofline"]; print("chunk '$c'", round(d["ms_per_step"],4), d["ms_per_step_each"][-3:], d.get("events_rounds_each")[-1], json.dumps({k: round(v,4) for k,v in r["device_ms_per_step_by_class"].items()}))'
done
