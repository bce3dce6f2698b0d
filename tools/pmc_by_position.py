"""Per-launch-position PMC table for one kernel (tools/pmc_gemm.sh output).

Dispatches of the kernel are numbered in order; position = index mod the
launches per forward (--per), so each row is one layer's launch averaged over
the forwards profiled.  usage: python tools/pmc_by_position.py gpurun_out/pmck --per 27
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--per", type=int, required=True)
a = ap.parse_args()
tab = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.root, "p*", "run_counter_collection.csv"))):
    disp = defaultdict(dict)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            d = int(row["Dispatch_Id"])
            disp[d][row["Counter_Name"]] = disp[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for i, d in enumerate(sorted(disp)):
        for c, v in disp[d].items():
            tab[i % a.per][c].append(v)
cols = sorted({c for p in tab.values() for c in p})
print("pos " + " ".join(f"{c[:24]:>24}" for c in cols))
for p in sorted(tab):
    vals = []
    for c in cols:
        v = tab[p].get(c)
        vals.append(f"{sum(v) / len(v):24.4g}" if v else " " * 24)
    print(f"{p:3d} " + " ".join(vals))
