"""Per-step durations of the one-reduction MGS sweep from a rocprofv3 kernel trace.

usage: python scripts/mgs_steps.py <kernel_trace.csv> <n> [iters]
Each solve runs steps k = 0..iters-1 in order; the k-th k_mgs1_dots / k_mgs1_update dispatch of a
solve is step k.  Algorithmic bytes per step:
  dots   (k+2)·8n   q_0..q_k and w
  update (k+4)·8n   q_0..q_k and w read, v written, q_k written back (pending normalisation)
Prints one JSON line per step: average µs and TB/s of both kernels.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = defaultdict(list)
    for r in rows:
        nm = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_mgs1_dots" in nm:
            seq["dots"].append(d)
        elif "k_mgs1_update" in nm:
            seq["update"].append(d)
    per = {kind: defaultdict(list) for kind in seq}
    for kind, ds in seq.items():
        for i, d in enumerate(ds):
            per[kind][i % iters].append(d)
    tot = {"dots": [0.0, 0.0], "update": [0.0, 0.0]}
    for k in range(iters):
        out = {"k": k}
        for kind, extra in (("dots", 2), ("update", 4)):
            v = per.get(kind, {}).get(k)
            if not v:
                continue
            us = sum(v) / len(v)
            by = (k + extra) * 8.0 * n
            out[kind + "_us"] = round(us, 2)
            out[kind + "_TBps"] = round(by / us / 1e6, 2)
            tot[kind][0] += us
            tot[kind][1] += by
        print(json.dumps(out))
    print(json.dumps({kind: {"us_per_solve": round(t[0], 1), "TBps": round(t[1] / t[0] / 1e6, 2) if t[0] else None}
                      for kind, t in tot.items()}))


if __name__ == "__main__":
    main()
