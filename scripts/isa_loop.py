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


def loop_census(lines, start, end):
    """Instruction classes summed over every block of the kernel that lies in a loop
    (label comment 'in Loop:' or 'Loop Header:'), by innermost loop header."""
    loops, cur = {}, None
    for ln in lines[start:end]:
        s = ln.strip()
        m = re.match(r"^(\.LBB\d+_\d+):.*(?:Header=(\S+)|Loop Header)", s)
        if re.match(r"^\.LBB\d+_\d+:", s):
            cur = None
            if m:
                cur = m.group(2) or m.group(1).lstrip(".")
                loops.setdefault(cur, [])
            continue
        if cur and s and not s.startswith((";", ".", "//")):
            loops[cur].append(cls(s))
    return loops


def main():
    path, kern = sys.argv[1], sys.argv[2]
    if "--loops" in sys.argv:
        lines = open(path).read().split("\n")
        start = next(i for i, ln in enumerate(lines) if ln.startswith("_Z") and kern in ln and ln.split(";")[0].rstrip().endswith(":"))
        end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
        for hdr, seq in loop_census(lines, start, end).items():
            seq = "".join(seq)
            print(kern, hdr, len(seq), {c: seq.count(c) for c in "MVTDSWNBGs"})
        return
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
