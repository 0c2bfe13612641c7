"""Instruction mix per basic block of one kernel in a hipcc -S listing (blocks with MFMAs or more
than N instructions): usage asm_blocks.py listing.s mangled-kernel-name [min-insts]"""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
minn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur, label = [], [], "entry"
for l in lines[start + 1:end]:
    s = l.strip()
    if re.match(r"^\.?L\w+:", s) or re.match(r"^\w+:", s):
        blocks.append((label, cur))
        label, cur = s.split(":")[0], []
        continue
    if not s or s.startswith((";", ".")):
        continue
    cur.append(s.split()[0])
blocks.append((label, cur))


def cat(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith(("ds_read", "ds_load")):
        return "ds_rd"
    if op.startswith(("ds_write", "ds_store")):
        return "ds_wr"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_st"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


for label, ops in blocks:
    c = Counter(cat(o) for o in ops)
    if c["mfma"] or len(ops) >= minn:
        print(f"{label:14s} n={len(ops):5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        if "-v" in sys.argv:
            print("   top valu:", Counter(o for o in ops if cat(o) == "valu").most_common(14))
