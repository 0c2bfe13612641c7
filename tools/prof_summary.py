"""Summarise a rocprofv3 kernel_stats.csv: per-step ms by kernel (steps = calls of a marker kernel)."""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
steps = next((int(r["Calls"]) for r in rows if marker in r["Name"]), 1)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"steps={steps} total/step={tot / steps / 1e6:.3f} ms")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:8.1f}us/step {float(r['Percentage']):5.1f}% "
          f"calls/step={int(r['Calls']) / steps:6.1f} avg={float(r['AverageNs']) / 1e3:7.1f}us  {r['Name'][:100]}")
