"""Per-leg roofline check against rocprofv3: for every leg profiled by tools/gpu_r06_prof.sh, the
bench's own JSON line of that run (trace_<leg>.json: the kernel(s) its roofline names, the launches it timed, the
algorithmic bytes per launch) and the kernel trace of the same run.  The dominant kernel's mean duration over its last
`launches` launches (the bench's instrumented steps come after its timed ones) gives the trace's fraction of the 8 TB/s
roofline; the bench's HIP-event fraction must agree within 3 %.  Also prints each leg's top kernels.

    python tools/leg_stats.py gpurun_out/r06/prof > profiles/r06/leg_roofline_vs_trace.txt
"""
import csv
import glob
import gzip
import json
import os
import re
import sys

PEAK = 8000.0
LEGS = ["c2", "c1", "c2s", "c3", "c4", "c4s", "c4c", "c5", "c5t"]


def norm(name):
    name = name.split("(")[0].replace("void ", "")
    for ns in ("scotty::", "kg::", "ck::", "wk::", "xq::", "ls::", "lc::", "ln::", "k::", "x::"):
        name = name.replace(ns, "")
    return name.replace(" ", "")


def roof_of(root, leg):
    try:
        line = open(os.path.join(root, "trace_%s.json" % leg)).read().strip().splitlines()[-1]
        d = json.loads(line)
    except (OSError, ValueError, IndexError):
        return None
    return d["roofline"] if leg == "c2" else (d.get("extra", {}).get(leg) or {}).get("roofline")


def main():
    root = sys.argv[1]
    for leg in LEGS:
        tr = glob.glob(os.path.join(root, "trace_" + leg, "**", "*kernel_trace.csv*"), recursive=True)
        st = glob.glob(os.path.join(root, "trace_" + leg, "**", "*kernel_stats.csv*"), recursive=True)
        op = lambda f: gzip.open(f, "rt") if f.endswith(".gz") else open(f)  # noqa: E731
        roof = roof_of(root, leg)
        if not tr or not roof:
            print("== %s: no trace / bench line" % leg)
            continue
        print("== %s" % leg)
        if st:
            rows = [r for r in csv.DictReader(op(st[0])) if "at::native" not in r["Name"]]
            rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
            for r in rows[:8]:
                print("  %-72s calls %6s  avg %9.1f us  total %8.2f ms" % (norm(r["Name"])[:72], r["Calls"],
                      float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
        trace = list(csv.DictReader(op(tr[0])))
        kn = roof.get("kernels") or [roof["kernel"]]
        kn = [norm(k) for k in kn]
        keep = int(roof.get("launches") or 1)
        algo = float(roof["algorithmic_bytes_per_launch"])
        if leg == "c4":  # the data pass: hist + scans + scatter + bucket per step
            kn = kn + ["scan_reduce_i32_kernel", "scan_small_i32_kernel", "scan_apply_i32_kernel"]
        total = 0.0
        for k in kn:
            t = sorted((r for r in trace if norm(r["Kernel_Name"]) == k), key=lambda r: int(r["Start_Timestamp"]))
            if not t:
                print("  (kernel %s not in the trace)" % k)
                continue
            last = t[-keep:]  # one launch per step (C4: the host-rows steps after the timed ones run the same pass)
            total += sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / keep
        if total <= 0:
            continue
        frac_trace = algo / total / PEAK  # bytes / ns = GB/s
        frac_bench = roof["frac"]
        print("  roofline kernel(s) %s: trace %.1f us/launch -> frac %.3f; bench (HIP events) frac %.3f; diff %.1f %%"
              % ("+".join(kn), total / 1e3, frac_trace, frac_bench, 100 * (frac_bench / frac_trace - 1)))


if __name__ == "__main__":
    main()
