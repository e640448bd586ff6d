"""Per-kernel launch statistics from a rocprofv3 kernel trace: the SQLite database (rocprofv3 -d DIR -o NAME, default
output) or a *_kernel_stats.csv.  Prints name, calls, average / total microseconds, sorted by total.  Host tool."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) "
                     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
                     "group by s.kernel_name").fetchall()
    return [(n, int(k), a / 1e3, t / 1e3) for n, k, a, t in rows]


def from_csv(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
    return out


def main():
    for arg in sys.argv[1:]:
        paths = glob.glob(os.path.join(arg, "**", "*.db"), recursive=True) if os.path.isdir(arg) else [arg]
        for p in paths:
            rows = from_db(p) if p.endswith(".db") else from_csv(p)
            rows.sort(key=lambda r: -r[3])
            print("# %s" % p)
            print("%-100s %7s %10s %12s" % ("kernel", "calls", "avg_us", "total_us"))
            for n, k, a, t in rows[:25]:
                print("%-100s %7d %10.1f %12.1f" % (n[:100], k, a, t))


if __name__ == "__main__":
    main()
