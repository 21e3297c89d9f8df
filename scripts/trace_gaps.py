"""Per-kernel launch gaps from a rocprofv3 kernel trace: for each kernel name, the mean idle time
between the end of the previous kernel on the same stream and its start, over the last N
dispatches (the timed steps).  Usage: trace_gaps.py <kernel_trace.csv> [N]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    rows = rows[-n:]
    last = {}
    gaps, durs = defaultdict(list), defaultdict(list)
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0].replace("void hgm::", "")[:60]
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]
        if q in last:
            gaps[nm].append((s - last[q]) / 1e3)
        last[q] = e
        durs[nm].append((e - s) / 1e3)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"span {span:.1f} us over {len(rows)} dispatches")
    for nm in sorted(durs, key=lambda k: -sum(durs[k])):
        g = gaps.get(nm, [0.0])
        print(f"{len(durs[nm]):5d} x {sum(durs[nm]) / len(durs[nm]):8.2f} us  gap before {sum(g) / len(g):6.2f} us  {nm}")


if __name__ == "__main__":
    main()
