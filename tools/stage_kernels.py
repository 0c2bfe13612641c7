"""Kernels of one replayed step between the stage marks (tsplat::stamp_kernel launches of
tools/graph_stages.py under rocprofv3 --kernel-trace): per segment between consecutive marks, the
kernel count, summed kernel time and the top kernels. Marks are numbered in trace order; the step is
the last complete one (segments of concurrent branches interleave, read the serial ones).
usage: stage_kernels.py run_results.db [--marks-per-step 32] [--top 6]"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--marks-per-step", type=int, default=32)
ap.add_argument("--top", type=int, default=6)
a = ap.parse_args()
rows = sorted(sqlite3.connect(a.db).execute("select name, start, end from kernels"), key=lambda r: r[1])
marks = [i for i, r in enumerate(rows) if "stamp_kernel" in r[0]]
if len(marks) < 2 * a.marks_per_step:
    raise SystemExit(f"only {len(marks)} marks")
step = marks[-a.marks_per_step:]  # the last step's marks (the replay loop ends the run)
for j in range(len(step) - 1):
    lo, hi = step[j], step[j + 1]
    seg = [r for r in rows[lo + 1:hi] if "stamp_kernel" not in r[0]]
    if not seg:
        continue
    tot = sum(e - s for _, s, e in seg) / 1e3
    agg = collections.Counter()
    cnt = collections.Counter()
    for n, s, e in seg:
        key = n.split("(")[0][:70]
        agg[key] += (e - s) / 1e3
        cnt[key] += 1
    print(f"--- mark {j} -> {j + 1}: {len(seg)} kernels, {tot:.1f} us busy")
    for k, t in agg.most_common(a.top):
        print(f"      {t:7.1f} us  x{cnt[k]:3d}  {k}")
