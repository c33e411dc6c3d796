#!/usr/bin/env python
"""Top kernels of a rocprofv3 --stats kernel_stats.csv, per step: python tools/kstats.py FILE [steps] [n]."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"total {tot / 1e6 / steps:.3f} ms/step over {calls / steps:.0f} launches/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    n = r["Name"]
    n = n if len(n) < 90 else n[:87] + "..."
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:7.1f}x "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {n}")
