"""HBM traffic of the C2 ingest kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
`bench.py --no-extra`, corrected per MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts a wide coalesced streaming read
at half its bytes: x2; WRITE_SIZE as is; both in kB) -> profiles/ingest_traffic.json, read by bench.py.

    python tools/ingest_traffic.py gpurun_out/pmc_ing_FETCH_SIZE gpurun_out/pmc_ing_WRITE_SIZE out.json
"""
import collections
import csv
import glob
import json
import os
import sys

BATCH = 1 << 27


def per_dispatch(d, counter):
    vals = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "ingest_kernel" not in r["Kernel_Name"]:
                continue
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")
    return vals, names


def main():
    fdir, wdir, out = sys.argv[1:4]
    f, names = per_dispatch(fdir, "FETCH_SIZE")
    w, _ = per_dispatch(wdir, "WRITE_SIZE")
    fk = sorted(f.values())[len(f) // 2]  # median launch (the timed steps; warm-up launches are smaller)
    wk = sorted(w.values())[len(w) // 2]
    algo = 12 * BATCH
    hbm = (2 * fk + wk) * 1024
    r = {"kernel": sorted(set(names.values()))[0], "batch": BATCH, "algorithmic_bytes_per_launch": algo,
         "FETCH_SIZE_kB_per_launch": fk, "WRITE_SIZE_kB_per_launch": wk,
         "correction": "gfx950: FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read "
                       "(MI355X_MICROARCH.md HBM) -> x2; WRITE_SIZE exact",
         "hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / algo,
         "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                   "python bench.py --no-extra --steps 3 --warmup 1 --no-cpu-baseline (median launch)"}
    json.dump(r, open(out, "w"), indent=1)
    print(json.dumps(r))


if __name__ == "__main__":
    main()
