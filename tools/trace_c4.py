"""Per-step kernel breakdown of the keyed (C4) leg from a rocprofv3 kernel trace: a step starts at kg_prep_kernel
(sort-free path) or key_insert_kernel (replay path); prints the last --steps steps.

    python tools/trace_c4.py gpurun_out/prof_c4/run_kernel_trace.csv
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "kg_prep_kernel" in r["Kernel_Name"]] or \
             [i for i, r in enumerate(rows) if "key_insert_kernel" in r["Kernel_Name"]]
    st = starts[-(args.steps + 1):]
    per, tot = collections.defaultdict(float), 0.0
    for a, b in zip(st[:-1], st[1:]):
        for r in rows[a:b]:
            if "at::native" in r["Kernel_Name"]:
                continue  # the bench's input generation, outside the timed region
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")[:60]] += d
            tot += d
    k = len(st) - 1
    print("scotty device time %.1f us/step over %d steps" % (tot / k, k))
    for name in sorted(per, key=lambda x: -per[x]):
        print("  %-60s %8.1f us/step" % (name, per[name] / k))


if __name__ == "__main__":
    main()
