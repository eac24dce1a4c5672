#!/usr/bin/env python3
"""Profiling-only: summarise a rocprofv3 kernel_trace.csv over the last FRACTION of its timeline
(the steady-state updates of a PPO probe): span, GPU-busy time (union of kernel intervals), and the
kernels by total time.  usage: trace_window.py <kernel_trace.csv> [fraction=0.4]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.4
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0, t1 = int(rows[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in rows)
    cut = t1 - (t1 - t0) * frac
    win = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
    busy, cs, ce = 0, None, None
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        a = agg[r["Kernel_Name"][:120]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"kernels {len(rows)}; window: last {frac:.0%} = {(t1 - cut) / 1e9:.3f} s, {len(win)} launches, "
          f"GPU busy {busy / 1e9:.3f} s, kernel sum {sum(v[1] for v in agg.values()) / 1e9:.3f} s")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{v[1] / 1e6:9.2f} ms {v[0]:6d} {v[1] / v[0] / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
