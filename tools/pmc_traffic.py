"""Digest rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic of one of
the hand-written kernels (MI355X_MICROARCH.md 'HBM' section: FETCH_SIZE and WRITE_SIZE come from
the L2's memory-side request counters, in KB; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced read, so it is doubled; WRITE_SIZE is exact for 16-B stores; Infinity-Cache hits
are counted, i.e. this is L2-miss traffic, an upper bound on HBM bytes).

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel-key> <out.json>
kernel-key selects dispatches whose name contains any of the comma-separated substrings; the
dispatches of one logical launch (e.g. attention + its combine) are summed per launch by
dividing by the number of dispatches of the FIRST substring."""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    out = defaultdict(float)
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out[r["Kernel_Name"]] += float(r["Counter_Value"])
        calls[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return out, {k: len(v) for k, v in calls.items()}


def main():
    fpath, wpath, key, out_path = sys.argv[1:5]
    keys = key.split(",")
    fetch, fcalls = load(fpath, "FETCH_SIZE")
    write, _ = load(wpath, "WRITE_SIZE")
    sel = lambda d: {k: v for k, v in d.items() if any(s in k for s in keys)}
    f_sel, w_sel = sel(fetch), sel(write)
    launches = max(n for k, n in fcalls.items() if keys[0] in k)
    fetch_b = 2 * 1024 * sum(f_sel.values()) / launches  # KB -> bytes, x2 gfx950 read correction
    write_b = 1024 * sum(w_sel.values()) / launches
    res = {"kernel_match": keys, "launches": launches, "fetch_bytes_per_launch": fetch_b,
           "write_bytes_per_launch": write_b, "traffic_bytes_per_launch": fetch_b + write_b,
           "kernels": sorted(f_sel), "source": [fpath, wpath],
           "note": "FETCH_SIZE x2 (gfx950 half-count of wide reads) + WRITE_SIZE, KB -> bytes"}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
