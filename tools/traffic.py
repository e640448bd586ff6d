"""HBM traffic per launch of each leg's measured kernels, from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
with per-access-pattern corrections calibrated on known-byte kernels (tools/pmc_calib.hip) -> profiles/traffic.json,
which bench.py reads only where the kernel names and the batch match the launches it timed.

    python tools/traffic.py calib <fetch_dir> <write_dir>                       # calibration (pmc_calib passes)
    python tools/traffic.py leg <leg> <batch> <fetch_dir> <write_dir> <kernel> [<kernel> ...]

Counters are in kB (rocprofv3); a kernel's value per launch is the median over its launches of at least half the
largest launch's bytes (warm-up steps with smaller batches drop out).  Correction per kernel: known bytes / counted
bytes of the calibration kernel with the same load (store) shape (PATTERN); WRITE_SIZE of a kernel whose stores are
not the scattered-run shape uses the coalesced-store factor.
"""
import collections
import csv
import glob
import gzip
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("TRAFFIC_OUT", os.path.join(ROOT, "profiles", "traffic.json"))

# kernel (normalised rocprof name prefix) -> (read calibration kernel, write calibration kernel)
PATTERN = {
    "ingest_kernel": ("calib_read16", "calib_write16"),
    "count_ingest_kernel": ("calib_read16", "calib_write16"),
    "kg_hist_kernel": ("calib_read16", "calib_write16"),
    "kg_scatter_kernel": ("calib_read_mix", "calib_write8_runs"),
    "kg_bucket_kernel": ("calib_read8", "calib_write8_runs"),
    "kg_bucket_mm_kernel": ("calib_read8", "calib_write8_runs"),
}


def norm(name):
    name = name.split("(")[0].replace("void ", "")
    for ns in ("scotty::", "kg::", "ck::", "wk::", "xq::", "ls::", "lc::", "ln::", "k::", "x::"):
        name = name.replace(ns, "")
    return name.replace(" ", "")


def per_kernel(d, counter):
    """{normalised kernel name: [kB per dispatch]} from a rocprofv3 counter-collection directory."""
    vals = collections.defaultdict(float)
    names = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv*"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under " + d)
    for f in files:
        fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] += float(r["Counter_Value"])
            names[key] = norm(r["Kernel_Name"])
    out = collections.defaultdict(list)
    for k, v in vals.items():
        out[names[k]].append(v)
    return out


def typical(xs):
    big = [x for x in xs if x >= 0.5 * max(xs)]
    return statistics.median(big)


def load():
    try:
        return json.load(open(OUT))
    except (OSError, ValueError):
        return {"legs": {}}


def calib(fdir, wdir):
    f, w = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    n = 1 << 26
    known_r = {"calib_read16": 16 * n, "calib_read_mix": 16 * n, "calib_read8": 8 * n, "calib_read4": 4 * n}
    known_w = {"calib_write8_runs": 8 * n, "calib_write16": 16 * n}
    fac = {}
    for k, b in known_r.items():
        fac[k] = {"known_bytes": b, "FETCH_SIZE_kB": typical(f[k]), "factor": b / (typical(f[k]) * 1024)}
    for k, b in known_w.items():
        fac[k] = {"known_bytes": b, "WRITE_SIZE_kB": typical(w[k]), "factor": b / (typical(w[k]) * 1024)}
    t = load()
    t["calibration"] = {"kernels": fac, "source": "tools/pmc_calib.hip under rocprofv3 --pmc FETCH_SIZE and, in a "
                                                  "separate pass, --pmc WRITE_SIZE (median of 3 launches each, every "
                                                  "launch behind a 1 GiB flush read)"}
    json.dump(t, open(OUT, "w"), indent=1)
    print(json.dumps(t["calibration"], indent=1))


def leg(name, batch, fdir, wdir, kernels):
    t = load()
    cal = t["calibration"]["kernels"]
    f, w = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    out = {}
    for k in kernels:
        kn = norm(k)
        if kn not in f or kn not in w:
            raise SystemExit("kernel %s not in the traces (have: %s)" % (kn, sorted(f)))
        base = kn.split("<")[0]
        # kernels without a calibrated shape of their own take the streaming one (every calibrated read factor is
        # 2.00 +- 0.01 and every write factor 1.00 on gfx950, profiles/traffic.json "calibration")
        rp, wp = PATTERN.get(base, ("calib_read16", "calib_write16"))
        fk, wk = typical(f[kn]), typical(w[kn])
        rb, wb = fk * 1024 * cal[rp]["factor"], wk * 1024 * cal[wp]["factor"]
        out[k] = {"FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk, "launches": len(f[kn]),
                  "read_pattern": rp, "read_factor": cal[rp]["factor"],
                  "write_pattern": wp, "write_factor": cal[wp]["factor"],
                  "read_bytes": rb, "write_bytes": wb, "hbm_bytes_per_launch": rb + wb}
    t["legs"][name] = {"batch": batch, "kernels": out,
                       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over python bench.py "
                                 "leg %s (typical launch), corrected by the calibration factors" % name}
    json.dump(t, open(OUT, "w"), indent=1)
    print(json.dumps(t["legs"][name], indent=1))


def all_legs(root):
    """Every leg profiled by tools/gpu_r06_prof.sh under root: the kernel names and batch from the bench line of the
    leg's own FETCH_SIZE run (its roofline block), then leg()."""
    if os.path.isdir(os.path.join(root, "calib_f")):  # else the calibration already in the output file
        calib(os.path.join(root, "calib_f"), os.path.join(root, "calib_w"))
    for f in sorted(glob.glob(os.path.join(root, "pmc_*_FETCH_SIZE.json"))):
        name = os.path.basename(f)[len("pmc_"):-len("_FETCH_SIZE.json")]
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            print("%s: no bench line" % name)
            continue
        roof = d["roofline"] if name == "c2" else (d.get("extra", {}).get(name) or {}).get("roofline")
        if not roof:
            continue
        kernels = roof.get("kernels") or [roof["kernel"]]
        batch = int(roof["algorithmic_bytes_per_launch"]) // (16 if name.startswith("c4") else 12)
        try:
            leg(name, batch, os.path.join(root, "pmc_%s_FETCH_SIZE" % name), os.path.join(root, "pmc_%s_WRITE_SIZE" % name),
                kernels)
        except (SystemExit, KeyError) as e:
            print("%s: %s" % (name, e))


if __name__ == "__main__":
    if sys.argv[1] == "calib":
        calib(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "all":
        all_legs(sys.argv[2])
    else:
        leg(sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5], sys.argv[6:])
