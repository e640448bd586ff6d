"""Per-step kernel breakdown from a rocprofv3 kernel trace (run_kernel_trace.csv).

A "step" of a grid-path leg starts at a cix_build_kernel launch (one per micro-batch).  Prints, for the last
--steps steps before the --leg-th grid-path operator boundary, every scotty kernel's average duration per step and
the step's summed device time.  Legs are separated where the ingest kernel's template changes or a gap of more than
--gap-ms seconds occurs between launches.

    python tools/trace_steps.py gpurun_out/prof_c2s/run_kernel_trace.csv --steps 5
"""
import argparse
import csv
import collections


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("scotty::", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--gap-ms", type=float, default=200.0)
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if "at::" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # split into legs at long idle gaps
    legs, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > args.gap_ms * 1e6 and cur:
            legs.append(cur)
            cur = []
        cur.append(r)
        last_end = e
    if cur:
        legs.append(cur)
    for li, leg in enumerate(legs):
        starts = [i for i, r in enumerate(leg) if "cix_build_kernel" in r["Kernel_Name"]] + [len(leg)]
        starts_all = starts[-(args.steps + 1):]
        if len(starts_all) < 2:
            continue
        per = collections.defaultdict(float)
        cnt = collections.defaultdict(int)
        total = 0.0
        nsteps = len(starts_all) - 1
        for a, b in zip(starts_all[:-1], starts_all[1:]):
            for r in leg[a:b]:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                per[short(r["Kernel_Name"])] += d
                cnt[short(r["Kernel_Name"])] += 1
                total += d
        span = (int(leg[starts_all[-1] - 1]["End_Timestamp"]) - int(leg[starts_all[0]]["Start_Timestamp"])) / 1e3
        print("leg %d: %d steps, device %.1f us/step, wall span %.1f us/step" % (li, nsteps, total / nsteps,
                                                                                span / nsteps))
        for k in sorted(per, key=lambda k: -per[k]):
            print("   %-50s %8.1f us/step  (%d launches)" % (k[:50], per[k] / nsteps, cnt[k]))


if __name__ == "__main__":
    main()
