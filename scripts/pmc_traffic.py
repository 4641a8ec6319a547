"""Per-launch HBM bytes of one kernel (or a '+'-joined group of kernels launched once
each per call, e.g. the two decoder attention backward kernels) from two rocprofv3
PMC passes.
usage: pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTRING[+SUBSTRING...] OUT_JSON"""
import csv
import json
import sys


def per_dispatch(d, counter, name):
    vals = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


fd, wd, name, out = sys.argv[1:5]
fetch_b = write_b = 0.0
parts, disp = {}, []
for k in name.split("+"):
    f = per_dispatch(fd, "FETCH_SIZE", k)
    w = per_dispatch(wd, "WRITE_SIZE", k)
    fb = 2.0 * 1024 * sum(f) / len(f)      # KB -> B, x2 for 16-B streaming reads on gfx950
    wb = 1024 * sum(w) / len(w)
    parts[k] = {"fetch_bytes": fb, "write_bytes": wb, "dispatches": [len(f), len(w)]}
    fetch_b += fb
    write_b += wb
    disp.append([len(f), len(w)])
res = {"kernel": name, "dispatches": disp, "fetch_bytes": fetch_b, "write_bytes": write_b,
       "traffic_bytes": fetch_b + write_b, "per_kernel": parts,
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py; "
                 "FETCH_SIZE x2 (gfx950 16-B read tally), KB -> bytes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
