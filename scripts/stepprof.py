"""Per-step kernel time by category from a rocprofv3 kernel trace, skipping the
warm-up steps (step boundaries = adamw_kernel dispatches).
    python scripts/stepprof.py gpurun_out/<run>_prof [--skip 1] [--top 25]"""
import argparse
import collections
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--skip", type=int, default=1)
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
rows = list(csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
start = ends[a.skip - 1] + 1 if a.skip > 0 else 0
sel = rows[start:ends[-1] + 1]
nsteps = len(ends) - a.skip


def cat(n):
    for key, c in (("gemm", "gemm"), ("splitk", "gemm"), ("attn_delta", "attn_delta"), ("dwf_", "dwconv"), ("dwb_", "dwconv"), ("dwb2_", "dwconv"),
                   ("dw_", "dwconv"), ("se_", "se"), ("bn_", "bn"), ("ln_", "ln"), ("gelu", "gelu"),
                   ("colsum", "colsum"), ("colred", "colsum"), ("im2col", "im2col"), ("col2im", "im2col"),
                   ("dropout", "dropout")):
        if key in n:
            return c
    if "attn" in n:
        return "attn_dec" if "<64" in n or "ILi64" in n else "attn_enc"
    return "other"


by_cat = collections.Counter()
by_k = collections.Counter()
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / nsteps
    by_cat[cat(r["Kernel_Name"])] += d
    by_k[r["Kernel_Name"][:90]] += d
tot = sum(by_cat.values())
print(f"{nsteps} steps, kernel time {tot:.1f} ms/step")
for k, v in by_cat.most_common():
    print(f"  {k:12s} {v:8.1f} ms  {100 * v / tot:5.1f}%")
for k, v in by_k.most_common(a.top):
    print(f"  {v:8.1f} ms  {k}")
