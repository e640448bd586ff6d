# the PCIe leg after C4 with the earlier legs' objects collected and torch's cache emptied first
set -o pipefail
out=gpurun_out/r06/${1:-p18}
mkdir -p $out
for legs in c4,pcie; do
  timeout -k 10 400 python -u bench.py --skip-headline --only $legs --no-cpu-baseline > $out/legs_$legs.json 2> $out/legs_$legs.err || exit $?
  python -c "import json; d=json.load(open('$out/legs_$legs.json'))['extra']['pcie_inclusive']; print('$legs', round(d['pinned']['ms_per_step'],2), round(d['pageable']['ms_per_step'],2))"
done
