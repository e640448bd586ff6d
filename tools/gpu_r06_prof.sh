#!/bin/bash
# Round-6 measurement campaign: for every bench leg, one rocprofv3 --output-format csv --kernel-trace --stats run and
# two --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs), plus the known-byte calibration kernels
# (tools/pmc_calib.hip).  Every step has its own time limit and the chain stops at the first failure.
# $1 = tag (output gpurun_out/r06/$1), $2 = legs (default: all), $3 = what (trace,pmc,calib; default all three)
set -o pipefail
tag=${1:-prof}
legs=${2:-"c2 c1 c2s c3 c4 c4s c4c c5 c5t"}
what=${3:-"calib,trace,pmc"}
out=gpurun_out/r06/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# keep what the analysis reads, compressed: gpurun copies back at most 64 MiB of gpurun_out
shrink() {
  find "$1" -type f ! -name "*.csv" ! -name "*.gz" -size +256k -delete 2>/dev/null
  find "$1" -type f -name "*.csv" -size +64k -exec gzip -9 {} \; 2>/dev/null
  du -sh "$1" | tail -1
}
args_of() {
  case $1 in
    c2) echo "--no-extra --no-cpu-baseline --steps 5 --warmup 2 --roof-steps 5" ;;
    *) echo "--skip-headline --no-cpu-baseline --only $1" ;;
  esac
}
if [[ $what == *calib* ]]; then
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $out/calib_f -o run -- ./tools/pmc_calib > $out/calib.json || exit 1
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $out/calib_w -o run -- ./tools/pmc_calib > /dev/null || exit 1
  shrink $out/calib_f; shrink $out/calib_w
  echo "calib done"
fi
for leg in $legs; do
  a=$(args_of $leg)
  if [[ $what == *trace* ]]; then
    timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --stats -d $out/trace_$leg -o run -- python3 -u bench.py $a \
      > $out/trace_$leg.json 2> $out/trace_$leg.err || { echo "trace $leg failed"; exit 1; }
    shrink $out/trace_$leg
    echo "trace $leg done"
  fi
  if [[ $what == *pmc* ]]; then
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 500 rocprofv3 --output-format csv --pmc $c -d $out/pmc_${leg}_$c -o run -- python3 -u bench.py $a \
        > $out/pmc_${leg}_$c.json 2> $out/pmc_${leg}_$c.err || { echo "pmc $leg $c failed"; exit 1; }
      shrink $out/pmc_${leg}_$c
    done
    echo "pmc $leg done"
  fi
done
du -sh $out
# the analysis on the box too (small outputs; the raw csv stay compressed under $out)
if [[ $what == *pmc* ]]; then
  TRAFFIC_OUT=$out/traffic.json python3 tools/traffic.py all $out > $out/traffic.txt 2>&1 || true
fi
if [[ $what == *trace* ]]; then
  python3 tools/leg_stats.py $out > $out/leg_roofline_vs_trace.txt 2>&1 || true
fi
