"""Before/after SQ-counter table from two scripts/pmc_kernel.sh-style pass sets:
    python scripts/pmc_ab_table.py gpurun_out/TAG_a gpurun_out/TAG_b KERNEL_FILTER[||FILTER_B] [label_a label_b]
Per dispatch: wave cycles, waits as a share of wave cycles, VALU / LDS / MFMA work."""
import collections
import csv
import glob
import sys


def load(tag, flt):
    v = collections.defaultdict(float)
    d = collections.defaultdict(set)
    for p in sorted(x for x in glob.glob(tag + "_p*") if not x.endswith(".log")):
        for r in csv.DictReader(open(p + "/run_counter_collection.csv")):
            if flt in r["Kernel_Name"]:
                v[r["Counter_Name"]] += float(r["Counter_Value"])
                d[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: v[k] / len(d[k]) for k in v}


a, b, flt = sys.argv[1], sys.argv[2], sys.argv[3]
la, lb = (sys.argv[4], sys.argv[5]) if len(sys.argv) > 5 else ("before", "after")
fa, fb = flt.split("||") if "||" in flt else (flt, flt)   # "A||B": different kernel names per arm
A, B = load(a, fa), load(b, fb)
rows = [("SQ_WAVE_CYCLES", None), ("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"), ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
        ("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"), ("SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
        ("SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"), ("SQ_VALU_MFMA_BUSY_CYCLES", None), ("SQ_BUSY_CYCLES", None),
        ("SQ_INSTS_VALU", None), ("SQ_INSTS_MFMA", None), ("SQ_INSTS_LDS", None), ("SQ_INSTS_SALU", None),
        ("SQ_LDS_BANK_CONFLICT", None)]
print(f"kernel filter: {flt}   (per dispatch; shares of SQ_WAVE_CYCLES in brackets)")
print(f"{'counter':28s} {la:>22s} {lb:>22s}   after/before")
for k, den in rows:
    if k not in A and k not in B:
        continue
    x, y = A.get(k, float('nan')), B.get(k, float('nan'))
    sx = f" ({x / A[den]:.1%})" if den and den in A and A[den] else ""
    sy = f" ({y / B[den]:.1%})" if den and den in B and B[den] else ""
    print(f"{k:28s} {x:12.4g}{sx:>10s} {y:12.4g}{sy:>10s}   {y / x if x else float('nan'):.3f}")
