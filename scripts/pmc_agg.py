"""Aggregate rocprofv3 --pmc counter CSVs per kernel (mean per dispatch)."""
import collections
import csv
import sys

for p in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0][-44:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        nd[k].add(r["Dispatch_Id"])
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].values())):
        n = len(nd[k])
        print(f"{k:44s} {n:4d} " + " ".join(f"{c[3:]}={x / n:.3g}" for c, x in sorted(v.items())))
