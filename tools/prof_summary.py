"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown.

usage: python tools/prof_summary.py <prof_dir> [steps | auto] > profiles/<name>.md
"""
import csv
import glob
import os
import sys


def main(d, steps=1):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(stats)))
    if steps == "auto":   # the capturable Adam's constants kernel runs once per C3 step
        steps = sum(int(r["Calls"]) for r in rows if "k_adam_consts" in r["Name"]) or 1
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# rocprofv3 kernel stats: {os.path.basename(stats)}\n")
    print(f"total kernel time {tot / 1e6:.2f} ms over the profiled run"
          + (f" ({tot / 1e6 / steps:.2f} ms per step, {steps} steps)" if steps > 1 else "") + "\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        print(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    arg = sys.argv[2] if len(sys.argv) > 2 else "1"
    main(sys.argv[1], arg if arg == "auto" else int(arg))
