"""Steady-state per-step kernel summary from a rocprofv3 kernel trace (run_kernel_trace.csv).

A step is the span between consecutive dispatches of a marker kernel that runs once per step
(default: the rasterizer's render_kernel, the last kernel of test_step). Only steps in the middle
of the run are averaged (the first `--skip` spans hold warmup, MIOpen's algorithm search and
graph capture; the last span holds the eager pass bench.py times the roofline kernel with), so
one-time work never lands in the per-step numbers.
usage: prof_steps.py run_kernel_trace.csv|run_results.db [--marker render_kernel] [--skip 4] [--top 40]
       [--timeline out.txt] [--grids substring]  (one steady-state step, every dispatch in start order with its queue and the
       idle time since the previous dispatch ended; rocprofv3's default SQLite output is read directly)"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="render_kernel")
ap.add_argument("--skip", type=int, default=4)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--timeline", default=None)
ap.add_argument("--grids", default=None, help="kernels whose name contains this: per-step time by launch grid")
a = ap.parse_args()
if a.trace.endswith(".db"):
    import sqlite3
    cur = sqlite3.connect(a.trace).execute("select name, start, end, queue_id, grid_x, grid_y, workgroup_x from kernels")
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Queue_Id": q,
             "Grid": f"{gx}x{gy}/{wx}"} for n, s, e, q, gx, gy, wx in cur]
else:
    rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [int(r["End_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
spans = list(zip(ends[a.skip:-2], ends[a.skip + 1:-1]))
if not spans:
    raise SystemExit(f"not enough '{a.marker}' dispatches ({len(ends)}) for steady-state spans")
tot = defaultdict(float)
cnt = defaultdict(int)
busy = 0.0
for lo, hi in spans:
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo < e <= hi:
            tot[r["Kernel_Name"]] += e - s
            cnt[r["Kernel_Name"]] += 1
            busy += e - s
n = len(spans)
wall = sum(hi - lo for lo, hi in spans) / n
print(f"steady-state steps averaged: {n}; wall per step {wall / 1e6:.3f} ms, kernel busy per step "
      f"{busy / n / 1e6:.3f} ms")
for name, t in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
    print(f"{t / n / 1e3:8.1f}us/step {t / busy * 100:5.1f}% calls/step={cnt[name] / n:6.1f} "
          f"avg={t / cnt[name] / 1e3:7.1f}us  {name[:100]}")
if a.timeline:
    lo, hi = spans[len(spans) // 2]
    step = [r for r in rows if lo < int(r["End_Timestamp"]) <= hi]
    with open(a.timeline, "w") as f:
        last_end = lo
        for r in step:
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            f.write(f"{(s0 - lo) / 1e3:9.1f} {(e0 - s0) / 1e3:7.1f} gap={(s0 - last_end) / 1e3:6.1f} "
                    f"q={r.get('Queue_Id', '?')} {r.get('Grid', '')} {r['Kernel_Name'][:110]}\n")
            last_end = max(last_end, e0)

if a.grids:
    def grid_of(r):
        if "Grid" in r:
            return r["Grid"]
        gx = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        return f"{gx}x{r.get('Grid_Size_Y', '?')}/{r.get('Workgroup_Size_X', r.get('Workgroup_Size', '?'))}"
    gt, gc = defaultdict(float), defaultdict(int)
    for lo, hi in spans:
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if lo < e <= hi and a.grids in r["Kernel_Name"]:
                key = (r["Kernel_Name"][:70], grid_of(r))
                gt[key] += e - s
                gc[key] += 1
    print(f"\nby grid ({a.grids}):")
    for key, t in sorted(gt.items(), key=lambda kv: -kv[1]):
        print(f"{t / n / 1e3:8.1f}us/step calls/step={gc[key] / n:5.1f} avg={t / gc[key] / 1e3:7.1f}us  grid={key[1]}  {key[0]}")
