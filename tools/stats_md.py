"""rocprofv3 --stats kernel summary (run_kernel_stats.csv) -> the markdown table
committed under profiles/.  usage: python tools/stats_md.py stats.csv "title" > out.md"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    print(f"## {title}\n")
    print("| kernel | calls | total us | avg us | share |")
    print("|---|---|---|---|---|")
    for r in rows:
        print(f"| `{r['Name']}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['Percentage']):.1f}% |")


if __name__ == "__main__":
    main()
