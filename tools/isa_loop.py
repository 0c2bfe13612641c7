"""Instruction classes per basic block of one kernel (device-only hipcc -S of a .hip source):
blocks with MFMAs, scratch traffic or AGPR copies. usage: isa_loop.py file.hip kernel-substring"""
import re
import subprocess
import sys
from pathlib import Path

root = Path(__file__).resolve().parents[1]
src, sub = sys.argv[1], sys.argv[2]
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-S", "--cuda-device-only",
                f"-I{root}/transplat_amd/csrc", f"-I{root}/include", src, "-o", "/tmp/_isa.s"], check=True,
               capture_output=True)
L = open("/tmp/_isa.s").read().splitlines()
names = [l.split(":")[0] for l in L if re.match(r"^_Z\w+:", l) and sub in l.split(":")[0]]
for name in names:
    st = next(i for i, l in enumerate(L) if l.startswith(name + ":"))
    en = next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
    print(name)
    blk, stats, order = "entry", {}, ["entry"]
    keys = ("v_mfma", "v_accvgpr_read", "v_accvgpr_write", "scratch_", "global_load", "ds_read", "ds_write",
            "s_barrier", "s_waitcnt", "v_exp")
    for l in L[st + 1:en]:
        s = l.strip()
        m = re.match(r"^(\.L\w+):", s)
        if m:
            blk = m.group(1)
            order.append(blk)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        d = stats.setdefault(blk, {"n": 0})
        d["n"] += 1
        for k in keys:
            if op.startswith(k):
                d[k] = d.get(k, 0) + 1
    for b in order:
        d = stats.get(b, {})
        if any(d.get(k) for k in ("v_mfma", "scratch_", "v_accvgpr_read", "v_accvgpr_write")):
            print(f"  {b:10s} " + " ".join(f"{k}={v}" for k, v in d.items()))
