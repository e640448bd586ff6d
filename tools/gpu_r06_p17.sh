# which earlier leg slows the PCIe-inclusive leg (14.4 ms alone, 17.8 ms at the end of the full bench)?
set -o pipefail
out=gpurun_out/r06/${1:-p17}
mkdir -p $out
for legs in c4,pcie c1,c2s,c3,pcie c4s,c4c,pcie c5,c5t,pcie; do
  timeout -k 10 400 python -u bench.py --skip-headline --only $legs --no-cpu-baseline > $out/legs_$legs.json 2> $out/legs_$legs.err || exit $?
  python -c "import json; d=json.load(open('$out/legs_$legs.json'))['extra']['pcie_inclusive']; print('$legs', round(d['pinned']['ms_per_step'],2), round(d['pageable']['ms_per_step'],2))"
done
