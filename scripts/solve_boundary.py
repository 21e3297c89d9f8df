"""Kernels between two solves of a bench trace (the setup and teardown of one solve): name, start
relative to the previous solve's last loop kernel, duration, stream.
usage: solve_boundary.py <kernel_trace.csv> <loop kernel substring> [n_before] [n_after]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    key = sys.argv[2]
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    na = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    # the biggest time gap between consecutive loop kernels marks a solve boundary
    gaps = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"]), a, b) for a, b in zip(idx[:-1], idx[1:])]
    _, a, b = max(gaps)
    t0 = int(rows[a]["End_Timestamp"])
    for r in rows[max(0, a - nb):min(len(rows), b + 2)][:nb + na]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  s{r['Stream_Id']}  {r['Kernel_Name'].split('(')[0][:70]}")


if __name__ == "__main__":
    main()
