"""Summarise rocprofv3 --pmc passes written by scripts/pmc_kernel.sh: per kernel
name, every counter of every pass summed over dispatches, and per dispatch.
    python scripts/pmc_sum.py gpurun_out/TAG [filter]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
res = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for d in sorted(p for p in glob.glob(tag + "_p*") if not p.endswith(".log")):
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        n = r["Kernel_Name"]
        if flt and flt not in n:
            continue
        res[n[:80]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n[:80]][r["Counter_Name"]].add(r["Dispatch_Id"])
for n, v in res.items():
    print(n)
    for k in sorted(v):
        nd = len(disp[n][k])
        print(f"    {k:28s} {v[k]:.4g}   ({nd} dispatches, {v[k] / nd:.4g} per dispatch)")
