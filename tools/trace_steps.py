"""Per-step kernel breakdown of a bench leg from a rocprofv3 kernel trace: a step starts at the kernel named by
--first (e.g. count_mark_kernel for the count path); the --steps longest steps are averaged.  Also prints the
step's span (first kernel start to last kernel end) so host gaps show as span - device time."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", required=True)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--median", action="store_true", help="average the --steps steps around the median instead")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "at::native" not in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(rows) if args.first in r["Kernel_Name"]] + [len(rows)]
    steps = []
    for a, b in zip(starts[:-1], starts[1:]):
        per = collections.defaultdict(float)
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")[:60]] += d
        span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
        steps.append((per, span))
    steps.sort(key=lambda p: -sum(p[0].values()))
    if args.median:
        m = len(steps) // 2
        sel = steps[max(0, m - args.steps // 2):max(0, m - args.steps // 2) + args.steps]
    else:
        sel = steps[:args.steps]
    tot = collections.defaultdict(float)
    for p, _ in sel:
        for k, v in p.items():
            tot[k] += v
    k = len(sel)
    print(("%d " + ("median" if args.median else "largest") + " steps: device %.1f us/step, span %.1f us/step") % (k, sum(tot.values()) / k,
                                                                       sum(s for _, s in sel) / k))
    for name in sorted(tot, key=lambda x: -tot[x]):
        print("  %-60s %8.1f us/step" % (name, tot[name] / k))


if __name__ == "__main__":
    main()
