# A/B of ingest variants (scotty_tune "ingest_mode" 0..3) and out-of-order fractions on the C2s workload
export TMPDIR=/tmp; mkdir -p gpurun_out
for m in ${MODES:-2 3}; do for o in ${OOOS:-0 0.02 0.2}; do
  echo "mode=$m ooo=$o" >> gpurun_out/ab_c2s.log
  timeout -k 10 100 python -u tools/perf_exact.py c2s --steps 5 --ooo $o --tune ingest_mode=$m >> gpurun_out/ab_c2s.log 2>&1 || exit 1
done; done
