"""Per-step kernel breakdown of the C3 leg (exact batch path) from a rocprofv3 kernel trace: a step starts at
xb_prep_kernel; the last --steps steps whose push carried the full batch (the longest steps) are printed."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "at::native" not in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(rows) if "xb_prep_kernel" in r["Kernel_Name"]] + [len(rows)]
    steps = []
    for a, b in zip(starts[:-1], starts[1:]):
        per = collections.defaultdict(float)
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")[:60]] += d
        steps.append(per)
    steps.sort(key=lambda p: -sum(p.values()))
    sel = steps[:args.steps]
    tot = collections.defaultdict(float)
    for p in sel:
        for k, v in p.items():
            tot[k] += v
    k = len(sel)
    print("C3: %d largest steps, device %.1f us/step" % (k, sum(tot.values()) / k))
    for name in sorted(tot, key=lambda x: -tot[x]):
        print("  %-60s %8.1f us/step" % (name, tot[name] / k))


if __name__ == "__main__":
    main()
