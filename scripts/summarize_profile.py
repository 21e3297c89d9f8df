"""Summarise rocprofv3 output of scripts/profile_bench.sh into profiles/.

Writes
  profiles/<tag>_<wl>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_<wl>_kernel_trace_summary.json  per-kernel avg duration from the trace
  profiles/traffic_<wl>.json             HBM bytes per launch per kernel class, from the
        FETCH_SIZE / WRITE_SIZE passes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
        The factor 2 is the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
        tallies 128-B requests at 64 B for coalesced streaming reads); it is applied to
        every kernel here, which over-states kernels that read with narrow scattered
        loads (calibrate before trusting an absolute for those).
Kernel classes: spmv_A_raymajor / spmv_B_pixelmajor are identified from the
problem's lanes-per-row template argument or the streaming/banded kernel names
(see DESIGN.md §3), mgs_pass_sweep = k_mgs_pass + k_mgs_normalize.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def classify(name, wl):
    if "k_mgs" in name:
        return "mgs_pass_sweep"
    if "k_spmv_stream" in name or "k_stream_fixup" in name or "k_spmv_band" in name or "k_band_reduce" in name:
        return "spmv_stream_or_band"
    if "k_spmv<" in name:
        g = name.split("k_spmv<")[1].split(",")[1].strip()
        if wl == "c2":
            return "spmv_A_raymajor" if g in ("32", "64") else "spmv_B_pixelmajor"
        return f"spmv_rows_G{g}"
    return None


def main():
    out, wl, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    prof = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "profiles"))
    os.makedirs(prof, exist_ok=True)
    st = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    if st:
        shutil.copy(st, os.path.join(prof, f"{tag}_{wl}_kernel_stats.csv"))
    tr = find(os.path.join(out, "trace", "**", "*kernel_trace.csv"))
    durs = defaultdict(list)
    if tr:
        for r in csv.DictReader(open(tr)):
            durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    summ = {k: {"calls": len(v), "avg_us": sum(v) / len(v), "total_us": sum(v)} for k, v in durs.items()}
    cls_dur = defaultdict(lambda: [0, 0.0])
    for k, v in summ.items():
        c = classify(k, wl)
        if c:
            cls_dur[c][0] += v["calls"]
            cls_dur[c][1] += v["total_us"]
    json.dump({"per_kernel": summ, "per_class": {c: {"calls": n, "avg_us": t / n} for c, (n, t) in cls_dur.items()}},
              open(os.path.join(prof, f"{tag}_{wl}_kernel_trace_summary.json"), "w"), indent=1)
    traffic = defaultdict(lambda: [0.0, 0])
    for pas, key in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = find(os.path.join(out, pas, "**", "*counter_collection.csv"))
        if not f:
            continue
        per = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != key:
                continue
            c = classify(r["Kernel_Name"], wl)
            if c:
                v = float(r["Counter_Value"]) * 1024.0 * (2.0 if key == "FETCH_SIZE" else 1.0)
                per[c].append(v)
        for c, vals in per.items():
            traffic[c][0] += sum(vals) / len(vals)
            traffic[c][1] = len(vals)
    res = {c: round(v[0]) for c, v in traffic.items()}
    json.dump(res, open(os.path.join(prof, f"traffic_{wl}.json"), "w"), indent=1)
    print(json.dumps({"traffic_bytes_per_launch": res,
                      "per_class_avg_us": {c: v[1] / v[0] for c, v in cls_dur.items()}}, indent=1))


if __name__ == "__main__":
    main()
