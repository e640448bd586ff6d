#!/bin/bash
# Grid-path parity, ingest A/B (mode 2 = per-lane slow path, 6 = deferred queue) on C2s, bench C2+C2s, rocprof.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/gpu_parity.log; exit 1; }
tail -2 gpurun_out/gpu_parity.log
: > gpurun_out/ab_c2s.log
for m in 2 6; do for o in 0 0.2; do
  echo "mode=$m ooo=$o" >> gpurun_out/ab_c2s.log
  timeout -k 10 120 python -u tools/perf_exact.py c2s --steps 5 --ooo $o --tune ingest_mode=$m >> gpurun_out/ab_c2s.log 2>&1 || { echo ab_failed; tail -20 gpurun_out/ab_c2s.log; exit 1; }
done; done
python3 - <<'PY'
import json
for line in open("gpurun_out/ab_c2s.log"):
    if line.startswith("mode="): tag=line.strip()
    elif line.startswith("{"):
        r=json.loads(line); ro=r["roofline"]
        print(tag, "ms/step %.3f ingest %.1f us frac %.3f frac_step %.3f classes %s" % (r["ms_per_step"], ro["avg_launch_ms"]*1e3, ro["frac"], ro["frac_step"], {k: round(v*1e3,1) for k,v in ro["device_ms_per_step_by_class"].items()}))
PY
timeout -k 10 400 python -u bench.py --no-cpu-baseline --only c2s > gpurun_out/bench_c2s.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench_c2s.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s -o run --output-format csv -- python -u bench.py --no-cpu-baseline --only c2s > gpurun_out/prof_c2s.log 2>&1 || { echo prof_failed; tail -5 gpurun_out/prof_c2s.log; exit 1; }
python3 tools/trace_steps.py gpurun_out/prof_c2s/run_kernel_trace.csv --steps 5
echo all_ok
