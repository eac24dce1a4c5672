#!/usr/bin/env python3
"""HBM traffic of the K-step rollout kernel (vss_rollout, bench.py's rollout leg) from two rocprofv3
--pmc passes, FETCH_SIZE and WRITE_SIZE, each in its own run (gfx950: the two cannot share a pass):

    python tools/rollout_pmc_summary.py <fetch run_counter_collection.csv> <write ...csv> <out.json>
        [--fields 65536] [--k 16] [--per-alloc 3]

Per launch: HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (the counters are KiB; gfx950's
FETCH_SIZE counts half of the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md §HBM,
tools/fetch_calib.hip), against the algorithmic bytes of bench.py's rollout_leg: fields x (K x 2,653 +
456).  The leg times its launches on several output allocations in turn (--per-alloc dispatches each:
one warm-up + the timed ones), so the launches are also grouped by allocation."""
import argparse
import collections
import csv
import json
import statistics


def per_dispatch(path, counter):
    by = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "rollout_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--fields", type=int, default=65536)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--per-alloc", type=int, default=3)
    a = ap.parse_args()
    fetch, write = per_dispatch(a.fetch, "FETCH_SIZE"), per_dispatch(a.write, "WRITE_SIZE")
    algo = a.fields * (a.k * 2653 + 456)
    n = min(len(fetch), len(write))
    rd = [2 * f * 1024 for f in fetch[:n]]
    wr = [w * 1024 for w in write[:n]]
    tot = [x + y for x, y in zip(rd, wr)]
    groups = [tot[i:i + a.per_alloc] for i in range(0, n, a.per_alloc)]
    res = {"kernel": "rollout_kernel", "fields": a.fields, "steps_per_launch": a.k, "launches": n,
           "algorithmic_bytes_per_launch": algo,
           "hbm_read_bytes_per_launch_mean": statistics.mean(rd), "hbm_write_bytes_per_launch_mean": statistics.mean(wr),
           "hbm_bytes_per_launch_mean": statistics.mean(tot),
           "traffic_over_algorithmic": statistics.mean(tot) / algo,
           "traffic_over_algorithmic_min": min(tot) / algo, "traffic_over_algorithmic_max": max(tot) / algo,
           "per_allocation_traffic_over_algorithmic": [round(statistics.mean(g) / algo, 4) for g in groups],
           "counters": "FETCH_SIZE x2 + WRITE_SIZE (KiB), separate rocprofv3 --pmc passes"}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
