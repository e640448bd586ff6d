#!/bin/bash
# Host-buffer ingest: parity of host pushes (pinned slots / pageable) + the PCIe-inclusive bench leg.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ingest_tests.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/ingest_tests.log; exit 1; }
tail -2 gpurun_out/ingest_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --only pcie --steps 3 --warmup 1 > gpurun_out/bench_pcie.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench_pcie.log; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/bench_pcie.log').read().strip().splitlines()[-1]); print(json.dumps(r['extra']['pcie_inclusive'], indent=1))"
echo ingest_ok
