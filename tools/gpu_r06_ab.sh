#!/bin/bash
# Round-6 A/B pass: validation tests of the changed paths, then the C4c replay-occupancy A/B and the host_spin A/B
# (C2 headline + C1 + C3, alternating runs on one box).  $1 = output tag; every GPU step has its own time limit.
set -o pipefail
out=gpurun_out/r06/${1:-ab}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keyed_count.py tests/test_gpu_exact.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -5 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python3 -u bench.py --skip-headline --no-cpu-baseline --only c4c,c4c6 > $out/ab_c4c_occ.json 2> $out/ab_c4c_occ.err \
  || { echo "c4c A/B failed"; exit 1; }
echo "c4c A/B done"
timeout -k 10 300 python3 -u bench.py --skip-headline --no-cpu-baseline --only c4s,c4s2 > $out/ab_c4s_occ.json 2> $out/ab_c4s_occ.err \
  || { echo "c4s A/B failed"; exit 1; }
echo "c4s A/B done"
for r in 1 2; do
  for t in none host_spin=1; do
    tune=""; [ $t != none ] && tune="--tune $t"
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --only c1,c3 --steps 20 $tune > $out/ab_spin_${t}_$r.json \
      2> $out/ab_spin_${t}_$r.err || { echo "spin A/B $t failed"; exit 1; }
    echo "spin A/B $t run $r done"
  done
done
