"""Per-dispatch PMC counters from rocprofv3 SQLite output (rocprofv3 --pmc ... -d DIR -o NAME): for every kernel whose
name contains argv[1], the mean over its dispatches of each counter (summed over instances), plus the mean duration.
Usage: python tools/pmc_db.py ingest_kernel DIR [DIR ...].  Host tool."""
import collections
import glob
import os
import sqlite3
import sys


def main():
    pat = sys.argv[1]
    for d in sys.argv[2:]:
        for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            c = sqlite3.connect(db)
            rows = c.execute(
                "select kd.id, s.kernel_name, kd.grid_size_x / kd.workgroup_size_x, kd.end - kd.start, p.name, sum(e.value) "
                "from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id "
                "join rocpd_kernel_dispatch kd on kd.event_id = e.event_id "
                "join rocpd_info_kernel_symbol s on kd.kernel_id = s.id group by kd.id, p.name").fetchall()
            agg = collections.defaultdict(lambda: collections.defaultdict(list))
            dur = collections.defaultdict(dict)
            for kid, name, grid, du, cn, v in rows:
                if pat not in name:
                    continue
                key = (name.split("(")[0].replace("void ", ""), grid)
                agg[key][cn].append(v)
                dur[key][kid] = du
            print("# %s" % db)
            for key in sorted(agg):
                ds = list(dur[key].values())
                print("%s grid %d: %d dispatches, avg %.1f us" % (key[0], key[1], len(ds), sum(ds) / len(ds) / 1e3))
                for cn in sorted(agg[key]):
                    xs = agg[key][cn]
                    print("    %-24s %.4g" % (cn, sum(xs) / len(xs)))


if __name__ == "__main__":
    main()
