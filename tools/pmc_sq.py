"""Summarise rocprofv3 SQ counter passes per (kernel, grid): stall breakdown and
instruction mix.  usage: python tools/pmc_sq.py <counter_collection.csv>... """
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for path in sys.argv[1:]:
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (row["Kernel_Name"][:60], row.get("Grid_Size", ""))
                acc[key][row["Counter_Name"]] += float(row["Counter_Value"])
                cnt[key][row["Counter_Name"]] += 1
    names = sorted({c for v in acc.values() for c in v})
    print("| kernel | grid | " + " | ".join(names) + " |")
    print("|---|---|" + "---|" * len(names))
    for key in sorted(acc):
        vals = []
        for c in names:
            n = cnt[key].get(c, 0)
            vals.append(f"{acc[key][c] / n:.3g}" if n else "-")
        print(f"| `{key[0]}` | {key[1]} | " + " | ".join(vals) + " |")


if __name__ == "__main__":
    main()
