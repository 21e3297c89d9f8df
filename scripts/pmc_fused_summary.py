"""Summarise the PMC passes of scripts/r3_pmc_fused.sh (rocprofv3 --pmc, one counter group per run)
for the one-pass kernels (k_fused_ab / k_fused_rw; PMC_KERNELS): per-launch averages of every counter, plus the ratios DESIGN.md
§3.5 quotes (wait / issue fractions of wave cycles, LDS bank-conflict share, HBM bytes per launch with
the gfx950 FETCH_SIZE x2 correction).
usage: python scripts/pmc_fused_summary.py <dir with p1..pN> [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


KERNELS = os.environ.get("PMC_KERNELS", "k_fused_ab,k_fused_rw").split(",")
REDUCE = "k_fused_reduce"


def main():
    d = sys.argv[1]
    vals = defaultdict(list)
    red = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)
        perr = defaultdict(float)
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if any(k in kn for k in KERNELS):
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            elif REDUCE in kn:
                perr[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), v in per.items():
            vals[name].append(v)
        for (_, name), v in perr.items():
            red[name].append(v)
    avg = {k: sum(v) / len(v) for k, v in vals.items() if v}
    ravg = {k: sum(v) / len(v) for k, v in red.items() if v}
    out = {"kernels": KERNELS, "launches": {k: len(v) for k, v in vals.items()}, "per_launch": avg,
           "reduce_per_launch": ravg}
    g = avg.get
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
            if g(k) is not None:
                out[k + "/SQ_WAVE_CYCLES"] = round(g(k) / g("SQ_WAVE_CYCLES"), 4)
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        out["SQ_LDS_BANK_CONFLICT/SQ_LDS_IDX_ACTIVE"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 4)
    if g("FETCH_SIZE") is not None:
        out["hbm_read_bytes"] = 2.0 * g("FETCH_SIZE") * 1024.0
    if g("WRITE_SIZE") is not None:
        out["hbm_write_bytes"] = g("WRITE_SIZE") * 1024.0
    # the whole pass (the partial reduction included): the bench line's roofline "traffic"
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        rf, rw = ravg.get("FETCH_SIZE", 0.0), ravg.get("WRITE_SIZE", 0.0)
        out["pass_hbm_bytes"] = (2.0 * (g("FETCH_SIZE") + rf) + g("WRITE_SIZE") + rw) * 1024.0
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")


if __name__ == "__main__":
    main()
