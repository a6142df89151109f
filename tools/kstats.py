#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per step: tools/kstats.py <csv> <n_steps> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows) / n / 1e6
print(f"kernel time per step: {tot:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    ms = float(r["TotalDurationNs"]) / n / 1e6
    print(f"{ms:7.3f} ms {int(r['Calls']) / n:5.1f}x {float(r['AverageNs']) / 1e3:8.1f}us "
          f"{100 * ms / tot:5.1f}% {r['Name'][:100]}")
