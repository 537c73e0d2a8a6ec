"""Per-kernel averages of every counter in DIR/pmc*/pmc_counter_collection.csv
(rocprofv3 --pmc passes): one row per kernel name, counters summed over the
dispatch's XCDs / SEs and averaged over the kernel's dispatches.
usage: pmc_table.py DIR"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "lnx::" not in k:
            continue
        short = (k[:k.rfind(">(") + 1] if ">(" in k else k.split("(")[0]).replace("lnx::", "").replace("void ", "")
        c = r["Counter_Name"]
        vals[short][c] += float(r["Counter_Value"])
        disp[short][c].add(r["Dispatch_Id"])
for k in sorted(vals):
    print(k)
    for c in sorted(vals[k]):
        n = max(len(disp[k][c]), 1)
        print(f"  {c:28s} {vals[k][c] / n:16.4g}")
