"""Per-leg kernel statistics from the round-end rocprofv3 runs (one run per bench leg, tools/gpu_r03_final_b.sh): the
top kernels of each leg's kernel_stats.csv, and the dominant kernel's mean duration over the leg's timed launches
recomputed from its kernel trace -- the number each BENCH roofline block divides the algorithmic bytes by.

    python tools/leg_stats.py gpurun_out/r03final > profiles/r03/leg_kernel_stats.txt
"""
import csv
import glob
import os
import sys

LEGS = {  # leg -> (dominant kernel name fragment, algorithmic bytes per launch, launches kept: the last k)
    "c2": ("ingest_kernel<0, 1, 6>", 12 * (1 << 27), 10),
    "c1": ("ingest_kernel<0, 1, 6>", 12 * (1 << 26), 5),
    "c2s": ("ingest_kernel<0, 1, 6>", 12 * (1 << 27), 5),
    "c3": ("ingest_kernel<0, 6, 7>", 12 * (1 << 26), 10),
    "c4": ("kg_hist_kernel|scan_reduce_i32|scan_small_i32|scan_apply_i32|kg_scatter_kernel|kg_bucket_kernel",
           16 * (1 << 26), 5),  # the keyed data pass (bench class "ingest"): the per-step sum of these
    "c5": ("count_ingest_kernel", 12 * (1 << 27), 5),
    "c5t": ("count_ingest_kernel", 12 * (1 << 26), 5),
}


def main():
    root = sys.argv[1]
    for leg, (frag, algo, keep) in LEGS.items():
        d = os.path.join(root, "prof_" + leg)
        st = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not st or not tr:
            print("%s: no profile" % leg)
            continue
        rows = list(csv.DictReader(open(st[0])))
        rows = [r for r in rows if "at::native" not in r["Name"] and "rocclr" not in r["Name"]]
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        print("== %s (%s)" % (leg, os.path.relpath(st[0], root)))
        for r in rows[:8]:
            print("  %-70s calls %5s  avg %9.1f us" % (r["Name"].split("(")[0][:70], r["Calls"],
                                                        float(r["AverageNs"]) / 1e3))
        trace = list(csv.DictReader(open(tr[0])))
        avg = 0.0
        for f in frag.split("|"):  # several fragments: one launch of each per step, summed
            t = sorted((r for r in trace if f in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
            if t:
                ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in t[-keep:]]
                avg += sum(ds) / len(ds)
        if avg > 0:
            print("  dominant %s: last %d launches avg %.1f us -> %.1f GB/s = %.3f of 8 TB/s (algorithmic %d B)"
                  % (frag, keep, avg / 1e3, algo / avg, algo / avg / 8000.0, algo))


if __name__ == "__main__":
    main()
