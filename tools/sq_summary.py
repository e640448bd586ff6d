"""Per-kernel averages of SQ counters from tools/gpu_c4_counters.sh passes (the C4 data-pass kernels and their
neighbours): wave-cycle shares (SQ_WAIT_ANY parked on s_waitcnt / barriers, SQ_WAIT_INST_ANY issue stalls,
SQ_ACTIVE_INST_ANY issuing), LDS bank-conflict share of LDS cycles, instructions per wave.

    python tools/sq_summary.py gpurun_out/r06/c4sq
"""
import collections
import csv
import glob
import gzip
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv*"), recursive=True):
        fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scotty::", "")
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return per, disp


def main():
    root = sys.argv[1]
    tot = collections.defaultdict(dict)
    ndisp = {}
    for sub in sorted(glob.glob(os.path.join(root, "sq*"))):
        if not os.path.isdir(sub):
            continue
        per, disp = load(sub)
        for k, v in per.items():
            n = len(disp[k])
            ndisp[k] = n
            for c, x in v.items():
                tot[k][c] = x / n
    for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0)):
        v = tot[k]
        if not any(s in k for s in ("kg_", "lane_wm", "scan_")):
            continue
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        print("== %s (%d dispatches)" % (k, ndisp.get(k, 0)))
        print("   waves %.0f  wave-cycles/wave %.0f  busy %.0f" % (v.get("SQ_WAVES", 0), wc / max(1, v.get("SQ_WAVES", 1)),
                                                                v.get("SQ_BUSY_CYCLES", 0)))
        print("   share of wave cycles: wait_any %.2f  wait_inst_any %.2f  active %.2f  wait_inst_lds %.2f" % (
            v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            v.get("SQ_WAIT_INST_LDS", 0) / wc))
        lds = v.get("SQ_LDS_IDX_ACTIVE", 0)
        print("   LDS: insts %.0f  bank-conflict cycles %.0f (%.2f of LDS-active %.0f)  active_inst_lds %.2f  "
              "active_inst_vmem %.2f" % (v.get("SQ_INSTS_LDS", 0), v.get("SQ_LDS_BANK_CONFLICT", 0),
                                         v.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0, lds,
                                         v.get("SQ_ACTIVE_INST_LDS", 0) / wc, v.get("SQ_ACTIVE_INST_VMEM", 0) / wc))
        print("   VMEM rd %.0f wr %.0f  VALU %.0f" % (v.get("SQ_INSTS_VMEM_RD", 0), v.get("SQ_INSTS_VMEM_WR", 0),
                                                   v.get("SQ_INSTS_VALU", 0)))


if __name__ == "__main__":
    main()
