"""Summarise the hot loop of a kernel in a hipcc -S dump (gfx950).

python scripts/isa_loop.py attn.s KERNEL_SUBSTRING [--seq]

Finds the kernel's largest basic block, counts instruction classes and (--seq)
prints one letter per instruction: M mfma, V valu, T transcendental, D ds_read,
S ds_write, W s_waitcnt, N s_nop, B barrier, G global/buffer, s salu.
"""
import re
import sys


def blocks(lines, start, end):
    cur, name = [], "entry"
    for ln in lines[start:end]:
        s = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            if cur:
                yield name, cur
            name, cur = s[:-1], []
        elif s and not s.startswith((";", ".", "//")):
            cur.append(s)
    if cur:
        yield name, cur


def cls(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
        return "T"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "D"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "S"
    if op.startswith("s_waitcnt"):
        return "W"
    if op.startswith("s_nop"):
        return "N"
    if op.startswith("s_barrier"):
        return "B"
    if op.startswith(("global_", "buffer_")):
        return "G"
    if op.startswith("v_"):
        return "V"
    return "s"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("_Z") and kern in ln and ln.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    name, body = max(blocks(lines, start, end), key=lambda b: len(b[1]))
    seq = "".join(cls(i) for i in body)
    counts = {c: seq.count(c) for c in "MVTDSWNBGs"}
    print(lines[start].split(":")[0], name, len(body), counts)
    if "--seq" in sys.argv:
        for i in range(0, len(seq), 100):
            print(seq[i:i + 100])


if __name__ == "__main__":
    main()
