"""Summarise a rocprofv3 kernel_stats.csv: python scripts/profsum.py DIR [N]"""
import csv
import sys
d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
import glob
import os
f = os.path.join(d, "run_kernel_stats.csv")
if not os.path.exists(f):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:n]:
    name = r['Name'].replace('(anonymous namespace)::', '').replace('_ZN12_GLOBAL__N_1', '')[:100]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>4} "
          f"avg {float(r['AverageNs'])/1e3:9.1f}us  {name}")
