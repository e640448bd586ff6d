"""Kernel / copy sequence of chosen steps from a rocprofv3 kernel(+memory-copy) trace, with the gap before each
launch: `python tools/step_gaps.py <trace dir> <first kernel of a step> <step> [<step> ...]`."""
import csv
import glob
import os
import sys


def main():
    d, first = sys.argv[1], sys.argv[2]
    steps = [int(x) for x in sys.argv[3:]] or [10]
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            r["Kernel_Name"] = "COPY %s %s" % (r.get("Direction", ""), r.get("Size", ""))
            rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    for k in steps:
        if k + 1 >= len(starts):
            continue
        prev = None
        tot = 0.0
        for r in rows[starts[k]:starts[k + 1]]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print("%8.1f gap %8.1f us  %s" % (gap, (e - s) / 1e3, r["Kernel_Name"].split("(")[0][-60:]))
            prev = e
        tot = (int(rows[starts[k + 1]]["Start_Timestamp"]) - int(rows[starts[k]]["Start_Timestamp"])) / 1e3
        print("step %d: %.1f us launch to launch\n" % (k, tot))


if __name__ == "__main__":
    main()
