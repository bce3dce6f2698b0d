"""Summarise rocprofv3 --pmc counter CSVs (tools/pmc_kernel.sh output):
per kernel, the mean of each counter over its dispatches."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void vox::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")
