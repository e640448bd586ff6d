"""Mean per-dispatch PMC counter values per kernel over rocprofv3 counter-collection directories (one pass per
directory), for the scotty kernels.  FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B:
/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3 section).

    python tools/pmc_summary.py gpurun_out/pmc_kg_FETCH_SIZE gpurun_out/pmc_kg_WRITE_SIZE ...
"""
import collections
import csv
import glob
import os
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(float)  # (dispatch, counter) -> summed over dimensions
            names = {}
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")
                if "at::" in name:
                    continue
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = name
            for (disp, cn), v in per.items():
                if cn == "FETCH_SIZE":
                    v *= 2
                vals[names[disp]][cn].append(v)
    for name in sorted(vals):
        cs = vals[name]
        parts = []
        for cn in sorted(cs):
            xs = cs[cn][-20:]  # the steady-state dispatches
            m = sum(xs) / len(xs)
            parts.append("%s=%.4g" % (cn, m))
        print("%-55s %s" % (name[:55], " ".join(parts)))


if __name__ == "__main__":
    main()
