"""Steady-state per-step kernel summary from a rocprofv3 kernel trace (run_kernel_trace.csv).

A step is the span between consecutive dispatches of a marker kernel that runs once per step
(default: the rasterizer's render_kernel, the last kernel of test_step). Only steps in the middle
of the run are averaged (the first `--skip` spans hold warmup, MIOpen's algorithm search and
graph capture; the last span holds the eager pass bench.py times the roofline kernel with), so
one-time work never lands in the per-step numbers.
usage: prof_steps.py run_kernel_trace.csv [--marker render_kernel] [--skip 4] [--top 40]"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="render_kernel")
ap.add_argument("--skip", type=int, default=4)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
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
