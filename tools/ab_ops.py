"""Compare per-op times of two `bench.py --dump-ops` logs (same plan).
usage: python tools/ab_ops.py a.log b.log [--kind gemmpipe]"""
import sys


def ops(path, kind):
    out = []
    for line in open(path):
        parts = line.split()
        if len(parts) > 3 and parts[1] == "us" and (kind is None or parts[2] == kind):
            out.append((float(parts[0]), " ".join(parts[2:])))
    return out


kind = sys.argv[sys.argv.index("--kind") + 1] if "--kind" in sys.argv else None
a, b = ops(sys.argv[1], kind), ops(sys.argv[2], kind)
ta = tb = 0.0
for (x, d), (y, _) in zip(a, b):
    ta += x
    tb += y
    print(f"{x:8.1f} {y:8.1f} {y / x:6.3f}  {d[:110]}")
print(f"total {ta:.1f} {tb:.1f} {tb / ta:.3f}")
