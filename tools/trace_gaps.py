#!/usr/bin/env python3
"""Idle gaps of the GPU in a rocprofv3 kernel trace (profiling tool): kernels in start order, the
time between one kernel's end and the next one's start, the largest gaps listed with the kernels around
them, and the busy / idle split per second of the run.

    python tools/trace_gaps.py <run_kernel_trace.csv> [top]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]) for r in rows)
    t0 = ev[0][0]
    gaps = []
    end = ev[0][1]
    busy = {}
    for i in range(1, len(ev)):
        s, e, n = ev[i]
        if s > end:
            gaps.append((s - end, (end - t0) / 1e9, ev[i - 1][2], n))
        sec = int((s - t0) / 1e9)
        busy[sec] = busy.get(sec, 0) + (e - max(s, end) if e > end else 0)
        end = max(end, e)
    print(f"kernels {len(ev)}, span {(end - t0) / 1e9:.3f} s, idle {sum(g[0] for g in gaps) / 1e9:.3f} s")
    for sec in sorted(busy):
        print(f"  second {sec}: busy {busy[sec] / 1e9:.3f} s")
    print("largest gaps (ms, at s, after -> before):")
    for g in sorted(gaps, reverse=True)[:top]:
        print(f"  {g[0] / 1e6:9.2f} ms at {g[1]:8.3f} s  {g[2]}  ->  {g[3]}")


if __name__ == "__main__":
    main()
