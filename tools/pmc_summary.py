#!/usr/bin/env python3
"""Summarise rocprofv3 output for the VSS step kernel into profiles/.

Inputs (from tools/gpu_check.sh): gpurun_out/prof_<tag>/run_kernel_stats.csv (kernel-trace
--stats) and gpurun_out/pmc_{fetch,write}_<tag>/run_counter_collection.csv (separate --pmc
passes: FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B: the counters are in KiB, and on
gfx950 FETCH_SIZE reports half of the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md §HBM), so it is doubled.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernel_substr):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel_substr in r["Kernel_Name"]:
            by[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--kernel", default="step_kernel<0, false>")
    ap.add_argument("--fields", type=int, default=65536)
    ap.add_argument("--mode", default="full")
    ap.add_argument("--algo-bytes", type=int, default=3101)
    ap.add_argument("--suffix", default="", help="pmc dir suffix, e.g. '_sa' for pmc_fetch_sa_<tag>")
    ap.add_argument("--stats-dir", default=None, help="kernel-trace dir name (default prof_<tag>)")
    ap.add_argument("--out", default="pmc_traffic.json")
    args = ap.parse_args()
    out_dir = os.path.join(REPO, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    g = os.path.join(REPO, "gpurun_out")
    import hashlib
    with open(os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_step.hip"), "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    res = {"tag": args.tag, "kernel": args.kernel, "fields": args.fields, "mode": args.mode, "source_sha": sha}

    sdir = args.stats_dir or f"prof_{args.tag}"
    stats = os.path.join(g, sdir, "run_kernel_stats.csv")
    trace = os.path.join(g, sdir, "run_kernel_trace.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, f"{args.tag}_{sdir.replace('_' + args.tag, '')}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            if args.kernel in r["Name"]:
                res["avg_ns"] = float(r["AverageNs"])
                res["calls"] = int(r["Calls"])
    if os.path.exists(trace):
        # the launches of this field count only (one 64-lane wave per 32 fields: grid = 2 x fields)
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))
             if args.kernel in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 2 * args.fields]
        if d:
            res["avg_ns"], res["calls"] = statistics.mean(d), len(d)
            res["avg_ns_source"] = f"{sdir}/run_kernel_trace.csv, grid {2 * args.fields}"
    fpath = os.path.join(g, f"pmc_fetch{args.suffix}_{args.tag}", "run_counter_collection.csv")
    wpath = os.path.join(g, f"pmc_write{args.suffix}_{args.tag}", "run_counter_collection.csv")
    if os.path.exists(fpath) and os.path.exists(wpath):
        fetch = counters(fpath, args.kernel)["FETCH_SIZE"]
        write = counters(wpath, args.kernel)["WRITE_SIZE"]
        res["fetch_size_kib_mean"] = statistics.mean(fetch)
        res["write_size_kib_mean"] = statistics.mean(write)
        res["hbm_read_bytes_per_launch"] = 2 * res["fetch_size_kib_mean"] * 1024
        res["hbm_write_bytes_per_launch"] = res["write_size_kib_mean"] * 1024
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
        res["algorithmic_bytes_per_launch"] = args.algo_bytes * args.fields
        res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"]
        for name, p in (("fetch", fpath), ("write", wpath)):
            rows = [r for r in csv.DictReader(open(p)) if args.kernel in r["Kernel_Name"]]
            with open(os.path.join(out_dir, f"{args.tag}_pmc_{name}_{args.mode}{args.suffix}.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
        with open(os.path.join(out_dir, args.out), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
