"""HBM traffic of the keyed (C4) data pass per step from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
`tools/c4_run.py`, per kernel and summed over the data pass (kg_hist, the partition scan, kg_scatter, kg_bucket --
the launches bench.py times as class "ingest"), corrected per MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts a wide
coalesced streaming read at half its bytes: x2; WRITE_SIZE as is; both in kB) -> profiles/keyed_traffic.json, read by
bench.py's C4 leg as roofline.traffic.

The x2 read correction is calibrated for 16-byte-per-lane streaming reads (kg_hist's key loads); kg_scatter reads
4- / 8-byte lanes and kg_bucket 8-byte records, for which the guide has no calibration, so the per-kernel table keeps
the raw counter values beside the corrected ones and the algorithmic bytes of each kernel.

    python tools/keyed_traffic.py gpurun_out/pmc_kg_FETCH_SIZE gpurun_out/pmc_kg_WRITE_SIZE out.json
"""
import collections
import csv
import glob
import json
import os
import sys

BATCH = 1 << 26
KEYS = 1 << 20
DATA_PASS = ("kg_hist_kernel", "scan", "kg_scatter_kernel", "kg_bucket")  # class "ingest" of the C4 leg
ALGO = {  # algorithmic bytes per launch of each data-pass kernel (int32 values, 8-byte compact records)
    "kg_hist_kernel": 4 * BATCH,                 # keys
    "kg_scatter_kernel": 16 * BATCH + 8 * BATCH,  # key + ts + value in, one 8-byte record out
    "kg_bucket": 8 * BATCH,                      # records in (the per-key partials out are per key, not per tuple)
}


def short(name):
    return name.split("(")[0].replace("void ", "").replace("scotty::", "").replace("kg::", "")


def per_kernel(d, counter):
    """{kernel: [value per dispatch]} (values summed over counter dimensions)."""
    per = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "scotty" not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
    out = collections.defaultdict(list)
    for disp in sorted(per, key=int):
        out[names[disp]].append(per[disp])
    return out


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else 0.0


def main():
    fdir, wdir, out = sys.argv[1:4]
    f = per_kernel(fdir, "FETCH_SIZE")
    w = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    step_hbm = 0.0
    for name in sorted(set(f) | set(w)):
        fk, wk = median(f.get(name, [])), median(w.get(name, []))
        hbm = (2 * fk + wk) * 1024
        algo = next((v for k, v in ALGO.items() if k in name), None)
        data_pass = any(k in name for k in DATA_PASS)
        kernels[name] = {"FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk, "hbm_bytes_corrected": hbm,
                         "hbm_bytes_raw": (fk + wk) * 1024, "algorithmic_bytes": algo,
                         "launches": max(len(f.get(name, [])), len(w.get(name, []))), "data_pass": data_pass}
        if data_pass:
            step_hbm += hbm  # one launch of each data-pass kernel per step
    algo_step = 16 * BATCH
    r = {"batch": BATCH, "keys": KEYS, "algorithmic_bytes_per_step": algo_step,
         "hbm_bytes_per_step": step_hbm, "traffic_over_algorithmic": step_hbm / algo_step,
         "kernels": kernels,
         "correction": "gfx950: FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read "
                       "(MI355X_MICROARCH.md HBM) -> x2 on every read; WRITE_SIZE as is",
         "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, python tools/c4_run.py 3 "
                   "(median launch per kernel; data pass = kg_hist + scans + kg_scatter + kg_bucket)"}
    json.dump(r, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in r.items() if k != "kernels"}))
    for name, v in kernels.items():
        print("%-60s fetch %10.0f kB  write %10.0f kB  corrected %.3g B  algo %s" % (
            name[:60], v["FETCH_SIZE_kB"], v["WRITE_SIZE_kB"], v["hbm_bytes_corrected"], v["algorithmic_bytes"]))


if __name__ == "__main__":
    main()
