"""Per-kernel mean of every collected counter over the dispatches of rocprofv3 --pmc runs.
Usage: pmc_kernels.py <dir> [<dir> ...]  (each dir holds one pass's *counter_collection.csv)"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    per = defaultdict(lambda: defaultdict(dict))   # kernel -> counter -> dispatch -> value
    for d in sys.argv[1:]:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                nm = r["Kernel_Name"].split("(")[0].replace("void hgm::", "")[:60]
                c = r["Counter_Name"]
                did = r["Dispatch_Id"]
                per[nm][c][did] = per[nm][c].get(did, 0.0) + float(r["Counter_Value"])
    for nm, cs in per.items():
        n = max(len(v) for v in cs.values())
        if n < 10:
            continue
        print(f"== {nm}  ({n} dispatches)")
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v.values()) / len(v):16.1f}")


if __name__ == "__main__":
    main()
