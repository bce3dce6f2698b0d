"""Summarise a rocprofv3 rocpd database (or kernel_stats.csv) into markdown:
per-kernel calls, total/avg duration, share, VGPRs.  Usage:
  python tools/rocpd_summary.py <run_results.db|kernel_stats.csv> [title]"""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = []
    q = ("select name, count(*), sum(duration), avg(duration), max(vgpr_count), "
         "max(accum_vgpr_count), max(lds_size) from kernels group by name "
         "order by sum(duration) desc")
    for name, n, tot, avg, vg, ag, lds in c.execute(q):
        rows.append((name, n, tot / 1e3, avg / 1e3, vg, ag, lds))
    return rows


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, "", "", ""))
    return rows


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    total = sum(r[2] for r in rows)
    print(f"## {title}\n")
    print("| kernel | calls | total us | avg us | share | vgpr | agpr | lds |")
    print("|---|---|---|---|---|---|---|---|")
    for name, n, tot, avg, vg, ag, lds in rows:
        print(f"| `{name}` | {n} | {tot:.1f} | {avg:.2f} | {100*tot/total:.1f}% | {vg} | {ag} | {lds} |")


if __name__ == "__main__":
    main()
