"""HBM bytes per launch of EVERY kernel of a step from the two rocprofv3 PMC passes
(FETCH_SIZE x2 per the gfx950 correction, + WRITE_SIZE), grouped by kernel name and
sorted by total bytes -- the measured-traffic column beside the ledger's algorithmic
bytes.  usage: pmc_table.py FETCH_DIR WRITE_DIR [TOP]"""
import csv
import sys
from collections import defaultdict


def per_name(d, counter):
    disp = defaultdict(float)
    name_of = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
        name_of[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = defaultdict(list)
    for k, v in disp.items():
        out[name_of[k]].append(v)
    return out


fd, wd = sys.argv[1:3]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
f, w = per_name(fd, "FETCH_SIZE"), per_name(wd, "WRITE_SIZE")
rows = []
for name in set(f) | set(w):
    fv, wv = f.get(name, []), w.get(name, [])
    fb = 2.0 * 1024 * sum(fv)
    wb = 1024.0 * sum(wv)
    n = max(len(fv), len(wv))
    rows.append((fb + wb, name, n, fb / max(len(fv), 1), wb / max(len(wv), 1)))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"{'total_GB':>9} {'n':>5} {'fetch_MB/l':>11} {'write_MB/l':>11}  kernel   (all launches: {tot / 1e9:.1f} GB)")
for t, name, n, fb, wb in rows[:top]:
    print(f"{t / 1e9:9.2f} {n:5d} {fb / 1e6:11.1f} {wb / 1e6:11.1f}  {name[:110]}")
