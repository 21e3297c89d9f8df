"""Summarise rocprofv3 output of scripts/profile_bench.sh into profiles/.

Writes
  profiles/<tag>_<wl>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_<wl>_kernel_trace_summary.json  per-kernel and per-class durations from the trace
  profiles/traffic_<wl>.json             HBM bytes per SpMV launch per class, from the
        FETCH_SIZE / WRITE_SIZE passes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
        The factor 2 is the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
        tallies 128-B requests at 64 B for coalesced streaming reads); it is applied to
        every kernel here, which over-states kernels that read with narrow scattered
        loads (calibrate before trusting an absolute for those).
Classes (what bench.py's HIP events bracket): one SpMV is a GROUP of
dispatches in stream order —
  * row kernel  k_spmv<T, G, ...>: one dispatch; A (ray-major) if G >= 16, else B;
  * streaming   k_spmv_stream (+ k_stream_fixup) (+ k_band_reduce): A if the group ends
    with the band reduction (only long-row operators are banded), else B;
  * banded      k_spmv_band + k_band_reduce: A.
  * fused       k_fused_ab + k_fused_reduce: spmv_AB_fused (round 3, fused.hip).
mgs_pass_sweep = every k_mgs_pass / k_mgs_normalize dispatch.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def groups(dispatches):
    """dispatches: [(dispatch_id, name, value)] in dispatch order -> [(cls, [values])]."""
    out = []
    i = 0
    while i < len(dispatches):
        _, nm, val = dispatches[i]
        if "k_fused_ab" in nm or "k_fused_rw" in nm:   # one pass A*(B*q): main kernel + partial reduction
            vals = [val]
            if i + 1 < len(dispatches) and "k_fused_reduce" in dispatches[i + 1][1]:
                vals.append(dispatches[i + 1][2])
                i += 1
            out.append(("spmv_AB_fused", vals))
            i += 1
        elif "k_mgs" in nm:
            out.append(("mgs_pass_sweep", [val]))
            i += 1
        elif "k_spmv<" in nm:
            g = int(nm.split("k_spmv<")[1].split(",")[1].strip())
            out.append(("spmv_A_raymajor" if g >= 16 else "spmv_B_pixelmajor", [val]))
            i += 1
        elif "k_spmv_stream" in nm or "k_spmv_band" in nm:
            vals = [val]
            j = i + 1
            while j < len(dispatches) and "k_stream_fixup" in dispatches[j][1]:
                vals.append(dispatches[j][2])
                j += 1
            banded = j < len(dispatches) and "k_band_reduce" in dispatches[j][1]
            if banded:
                vals.append(dispatches[j][2])
                j += 1
            out.append(("spmv_A_raymajor" if banded or "k_spmv_band" in nm else "spmv_B_pixelmajor", vals))
            i = j
        else:
            i += 1
    return out


def traffic_of(dirs):
    """{class: HBM bytes per launch} from FETCH_SIZE / WRITE_SIZE counter passes (dirs: key -> dir)."""
    traffic = defaultdict(float)
    for key, d in dirs.items():
        f = find(os.path.join(d, "**", "*counter_collection.csv"))
        if not f:
            continue
        per_dispatch = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != key:
                continue
            did = int(r["Dispatch_Id"])
            v = float(r["Counter_Value"]) * 1024.0 * (2.0 if key == "FETCH_SIZE" else 1.0)
            nm, acc = per_dispatch.get(did, (r["Kernel_Name"], 0.0))
            per_dispatch[did] = (nm, acc + v)
        seqc = [(d_, nm, v) for d_, (nm, v) in sorted(per_dispatch.items())]
        per = defaultdict(list)
        for cls, vals in groups(seqc):
            per[cls].append(sum(vals))
        for cls, vals in per.items():
            traffic[cls] += sum(vals) / len(vals)
    return {c: round(v) for c, v in traffic.items()}


def main():
    if sys.argv[1] == "--traffic":      # scripts/gpu.sh traffic: <dir with FETCH_SIZE/ WRITE_SIZE/> <wl>
        d = sys.argv[2]
        print(json.dumps(traffic_of({k: os.path.join(d, k) for k in ("FETCH_SIZE", "WRITE_SIZE")}), indent=1))
        return
    out, wl, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    prof = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "profiles"))
    os.makedirs(prof, exist_ok=True)
    st = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    if st:
        import shutil
        shutil.copy(st, os.path.join(prof, f"{tag}_{wl}_kernel_stats.csv"))
    tr = find(os.path.join(out, "trace", "**", "*kernel_trace.csv"))
    durs = defaultdict(list)
    seq = []
    if tr:
        rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            durs[r["Kernel_Name"]].append(d)
            seq.append((int(r["Dispatch_Id"]), r["Kernel_Name"], d))
    summ = {k: {"calls": len(v), "avg_us": sum(v) / len(v), "total_us": sum(v)} for k, v in durs.items()}
    cls_dur = defaultdict(list)
    for cls, vals in groups(seq):
        cls_dur[cls].append(sum(vals))
    per_class = {c: {"calls": len(v), "avg_us": sum(v) / len(v)} for c, v in cls_dur.items()}
    json.dump({"per_kernel": summ, "per_class": per_class},
              open(os.path.join(prof, f"{tag}_{wl}_kernel_trace_summary.json"), "w"), indent=1)
    res = traffic_of({"FETCH_SIZE": os.path.join(out, "fetch"), "WRITE_SIZE": os.path.join(out, "write")})
    json.dump(res, open(os.path.join(prof, f"traffic_{wl}.json"), "w"), indent=1)
    print(json.dumps({"traffic_bytes_per_launch": res,
                      "per_class_avg_us": {c: v["avg_us"] for c, v in per_class.items()}}, indent=1))


if __name__ == "__main__":
    main()
