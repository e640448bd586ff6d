# A/B of ingest variants on the C2s workload (tools/perf_exact.py); modes >= 6 are timing probes only
export TMPDIR=/tmp; mkdir -p gpurun_out
for m in ${MODES:-2 6 10 14}; do
  echo "mode=$m" >> gpurun_out/ab_c2s.log
  timeout -k 10 100 python -u tools/perf_exact.py c2s --steps 5 --tune ingest_mode=$m >> gpurun_out/ab_c2s.log 2>&1 || exit 1
done
