"""Per-step overlap of concurrent branches from a rocprofv3 kernel trace (--kernel-trace csv):
steady-state steps are delimited by consecutive raster render launches; for each step, the wall
time, the union of kernel-busy intervals, the sum of kernel durations (> union when branches
overlap), and the busy time per hardware queue. Usage: python tools/overlap_report.py trace.csv"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    marks = [s for s, e, n, q in ev if "render_kernel" in n]
    steps = []
    for a, b in zip(marks[:-1], marks[1:]):
        ks = [(s, e, n, q) for s, e, n, q in ev if a < s <= b]
        if not ks:
            continue
        iv = sorted((s, e) for s, e, _, _ in ks)
        union, cur_s, cur_e = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > cur_e:
                union += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        union += cur_e - cur_s
        per_q = defaultdict(int)
        for s, e, _, q in ks:
            per_q[q] += e - s
        steps.append((b - a, union, sum(e - s for s, e, _, _ in ks), dict(per_q), len(ks)))
    steps = steps[len(steps) // 3:]  # drop warm-up
    n = len(steps)
    avg = lambda i: sum(s[i] for s in steps) / n / 1e3
    print(f"steady steps {n}: wall {avg(0):.1f} us, busy union {avg(1):.1f} us, kernel sum {avg(2):.1f} us, "
          f"launches {steps[-1][4]}")
    qs = defaultdict(int)
    for s in steps:
        for q, t in s[3].items():
            qs[q] += t
    print("per queue busy (us/step):", {q: round(t / n / 1e3, 1) for q, t in sorted(qs.items())})


if __name__ == "__main__":
    main(sys.argv[1])
