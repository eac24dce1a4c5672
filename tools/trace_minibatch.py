#!/usr/bin/env python3
"""Profiling-only: the kernels of one repeating window of a rocprofv3 kernel trace, in start order, with
their durations and the idle gap before each -- e.g. one update minibatch (from one launch of a marker
kernel to the next):

    python tools/trace_minibatch.py <run_kernel_trace.csv> <marker substring> [occurrence] [out.txt]

prints the window that starts at the marker's `occurrence`-th launch (default: the middle one), and a
per-kernel-name summary of that window (count, total us)."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker = sys.argv[2]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [i for i, e in enumerate(ev) if marker in e[2]]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) // 2
    a, b = starts[k], starts[k + 1]
    out = open(sys.argv[4], "w") if len(sys.argv) > 4 else sys.stdout
    span = (ev[b][0] - ev[a][0]) / 1e3
    busy = sum(e[1] - e[0] for e in ev[a:b]) / 1e3
    print(f"window: launches {b - a}, span {span:.1f} us, kernel time {busy:.1f} us, idle {span - busy:.1f} us", file=out)
    by = collections.defaultdict(lambda: [0, 0.0])
    prev_end = ev[a][0]
    for s, e, n in ev[a:b]:
        print(f"  {(s - prev_end) / 1e3:8.1f} gap  {(e - s) / 1e3:9.1f} us  {n[:110]}", file=out)
        prev_end = max(prev_end, e)
        by[n[:110]][0] += 1
        by[n[:110]][1] += (e - s) / 1e3
    print("by kernel (count, us):", file=out)
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"  {c:4d} {t:9.1f}  {n}", file=out)


if __name__ == "__main__":
    main()
