"""Compare per-op-kind totals of bench.py --dump-ops stderr dumps: ops_compare.py a.txt b.txt ..."""
import sys
from collections import defaultdict


def load(p):
    out = defaultdict(float)
    for line in open(p):
        line = line.strip()
        if " us " in line:
            t, rest = line.split(" us ", 1)
            out[rest.split()[0]] += float(t)
    return out


runs = [load(p) for p in sys.argv[1:]]
keys = sorted(set().union(*runs), key=lambda k: -runs[0].get(k, 0))
for k in keys:
    print(f"{k:12s}" + "".join(f" {r.get(k, 0):9.1f}" for r in runs))
print(f"{'total':12s}" + "".join(f" {sum(r.values()):9.1f}" for r in runs))
