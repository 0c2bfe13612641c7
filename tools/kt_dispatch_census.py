"""Per-dispatch census of a rocprofv3 --kernel-trace CSV: kernels grouped by (name, grid, workgroup)
with call counts and average durations, sorted by total time (which launch shapes the glue and the
direct convolutions come from). Usage: python tools/kt_dispatch_census.py <trace dir> [filter ...]"""
import collections
import csv
import glob
import sys

path = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
filters = sys.argv[2:]
cnt = collections.Counter()
tot = collections.defaultdict(float)
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if filters and not any(f in n for f in filters):
        continue
    k = (n[:70], r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Grid_Size_Y", ""), r.get("Workgroup_Size_X", ""))
    cnt[k] += 1
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k in sorted(cnt, key=lambda k: -tot[k]):
    print(f"{cnt[k]:4d} {tot[k] / cnt[k]:7.1f} us  {tot[k]:8.1f} us total  grid {k[1]} x {k[2]}  wg {k[3]}  {k[0]}")
