"""Median gap between consecutive kernels on the main queue of a rocprofv3 kernel trace.
usage: python scripts/trace_gaps.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
q = collections.Counter(r["Queue_Id"] for r in rows if "k_spmv" in r["Kernel_Name"]).most_common(1)[0][0]
main = [r for r in rows if r["Queue_Id"] == q]
short = lambda r: r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("hgm::", "")  # noqa: E731
gaps = collections.defaultdict(list)
for a, b in zip(main, main[1:]):
    gaps[(short(a), short(b))].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
for k, v in sorted(gaps.items(), key=lambda x: -len(x[1]))[:10]:
    v.sort()
    print(f"{k[0]:>16} -> {k[1]:<16} n={len(v):4d} median {v[len(v) // 2]:7.2f} us  p10 {v[len(v) // 10]:6.2f}")
durs = collections.defaultdict(list)
for r in main:
    durs[short(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
print({k: round(sorted(v)[len(v) // 2], 2) for k, v in durs.items() if len(v) > 20})
