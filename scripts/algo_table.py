"""Algorithmic roofline fraction per kernel family of one bench step, from a
per-op ledger (scripts/ledger.py output, e.g. profiles/r02v_ledger.txt).

Work is ALGORITHMIC: GEMM 2*M*N*K per product; attention
forward 4*B*H*L^2*D, backward 8*B*H*L^2*D (2x forward: dV, dP, dQ, dK -- the
recompute of S/P that flash kernels execute is not counted); streaming ops
their tensor bytes (every distinct argument/output once, as the ledger counts
them).  MFMA families are priced against 2.5 PF dense bf16, streaming families
against 8 TB/s.  The kernel_stats CSV of the same tree (rocprofv3 --stats) is
used to cross-check the attention families, whose kernel names are unique.

    python scripts/algo_table.py profiles/r02v_ledger.txt [profiles/r02v_kernel_stats.csv STEPS]

STEPS = the steps the CSV's trace holds, warm-up included (r02_measure.sh: 1 + 3).
"""
import csv
import re
import sys

MFMA = 2.5e15
HBM = 8.0e12
ROW = re.compile(r"^\s*(-?[\d.]+)\s+([\d.]+)\s+([\d.]+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(\S+)\s*(.*)$")
TENS = re.compile(r"(\w+)\[([\d, ]+)\]")
INTS = re.compile(r"\b(\w+)=(\d+)")


def shapes(s):
    return {n: [int(v) for v in d.split(",")] for n, d in TENS.findall(s)}


def classify(op, sh, kv):
    """-> (family, flop, bound)"""
    if op in ("attn_fwd", "attn_bwd"):
        N, L, H, D = kv["N"], kv["L"], kv["H"], kv["D"]
        f = (4.0 if op == "attn_fwd" else 8.0) * N * H * L * L * D
        who = "decoder" if D == 64 else f"encoder L={L}"
        return f"attention {who} {'fwd' if op == 'attn_fwd' else 'bwd'}", f, "mfma"
    if op in ("linear", "linear_bn_stats", "linear_se"):
        x = sh.get("x") or sh.get("a2")
        w = sh["w"]
        fam = "stem conv1 (GEMM)" if w[0] == 48 else "GEMM fwd"
        return fam, 2.0 * x[0] * x[1] * w[0], "mfma"
    if op == "linear_dx":
        dy, w = sh["dy"], sh["w"]
        return "GEMM dX", 2.0 * dy[0] * dy[1] * w[1], "mfma"
    if op.startswith("linear_dw"):
        dy = sh["dy"]
        x = sh.get("x") or sh.get("a2")
        fam = "stem conv1 (GEMM)" if dy[1] == 48 else "GEMM dW"
        return fam, 2.0 * dy[0] * dy[1] * x[1], "mfma"
    if op.startswith("conv3x3") or op == "stem_im2col":
        return "stem conv2 / im2col", 0.0, "hbm"
    if op.startswith("dwconv") or op.startswith("se_"):
        st0 = any(v[0] == 25690112 for v in sh.values())
        return "MBConv streaming (stage 0, 112^2)" if st0 else "MBConv streaming (56^2 / 28^2)", 0.0, "hbm"
    return "other streaming (LN, BN, dropout, blend, loss, AdamW)", 0.0, "hbm"


def main():
    led = sys.argv[1]
    fam = {}
    step_ms = ops_ms = None
    for line in open(led):
        if line.startswith("step "):
            m = re.findall(r"([\d.]+) ms", line)
            step_ms, ops_ms = float(m[0]), float(m[1])
            continue
        m = ROW.match(line)
        if not m:
            continue
        ms, n, gbs = float(m.group(2)), int(m.group(4)), float(m.group(5))
        op, rest = m.group(7), m.group(8)
        sh = shapes(rest)
        kv = {k: int(v) for k, v in INTS.findall(rest)}
        name, flop, bound = classify(op, sh, kv)
        nbytes = gbs * 1e6 * ms          # ledger GB/s = bytes / ms / 1e6
        g = fam.setdefault(name, [0.0, 0.0, 0.0, bound, 0])
        g[0] += ms
        g[1] += flop * n                 # shapes are per call; the row sums n calls
        g[2] += nbytes
        g[4] += n
    listed = sum(g[0] for g in fam.values())
    print(f"source: {led}; step {step_ms} ms, ops {ops_ms} ms, ledger rows listed {listed:.1f} ms")
    print(f"{'family':52s} {'ms/step':>8s} {'launch':>6s} {'algo work':>12s} {'achieved':>12s} {'frac':>6s}")
    for name, (ms, flop, nb, bound, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        if bound == "mfma":
            a = flop / (ms * 1e-3)
            print(f"{name:52s} {ms:8.1f} {n:6d} {flop / 1e12:9.2f} TF {a / 1e12:8.1f} TF/s {a / MFMA:6.3f}")
        else:
            a = nb / (ms * 1e-3)
            print(f"{name:52s} {ms:8.1f} {n:6d} {nb / 1e9:9.1f} GB {a / 1e9:8.0f} GB/s {a / HBM:6.3f}")
    if ops_ms:
        print(f"{'(ops not in the listed rows)':52s} {ops_ms - listed:8.1f}")
    if len(sys.argv) > 3:
        csvf, steps = sys.argv[2], int(sys.argv[3])
        tot = {}
        for r in csv.DictReader(open(csvf)):
            nm = r["Name"]
            for key, pat in (("attention decoder bwd", r"attn_bwd_(dq|dkdv)(16)?_bf16<64"),
                             ("attention decoder fwd", r"attn_fwd_bf16<64"),
                             ("attention encoder bwd (both L)", r"attn_bwd_(dq|dkdv)(16)?_bf16<32"),
                             ("attention encoder fwd (both L)", r"attn_fwd_bf16<32")):
                if re.search(pat, nm):
                    tot[key] = tot.get(key, 0.0) + float(r["TotalDurationNs"]) / 1e6 / steps
        print(f"\ncross-check from {csvf} ({steps} steps, rocprofv3 kernel time per step):")
        for k, v in tot.items():
            print(f"  {k:40s} {v:8.1f} ms/step")


if __name__ == "__main__":
    main()
