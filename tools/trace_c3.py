"""Per-step kernel breakdown of the C3 leg (exact batch path) from a rocprofv3 kernel trace: a step (one push
round) starts at xb_prep_kernel.  Prints the median round (the steady state) and the largest one (a pause step
with many events and apply segments)."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="xq_prep_kernel", help="kernel that starts a step (xb_prep_kernel: the "
                    "event-exact path's round)")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "at::native" not in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]] + [len(rows)]
    steps, spans, calls = [], [], []
    for a, b in zip(starts[:-1], starts[1:]):
        per = collections.defaultdict(float)
        cnt = collections.Counter()
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")[:60]
            per[k] += d
            cnt[k] += 1
        steps.append(per)
        calls.append(cnt)
        spans.append((int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    order = sorted(range(len(steps)), key=lambda i: sum(steps[i].values()))
    for label, i in (("median", order[len(order) // 2]), ("largest", order[-1])):
        p = steps[i]
        print("C3 %s step of %d: device %.1f us, first start to last end %.1f us, %d launches" %
              (label, len(steps), sum(p.values()), spans[i], sum(calls[i].values())))
        for name in sorted(p, key=lambda x: -p[x])[:14]:
            print("  %-60s %8.1f us  %4d calls" % (name, p[name], calls[i][name]))


if __name__ == "__main__":
    main()
