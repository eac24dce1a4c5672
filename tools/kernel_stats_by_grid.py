#!/usr/bin/env python3
"""rocprofv3 kernel-trace summary split per (kernel, grid size): rocprofv3's own --stats file averages
every launch of a kernel name together, so a command that launches one kernel at several sizes (the
bench's FULL step at 65,536 and at 131,072 fields) cannot be read from it per size.

    python tools/kernel_stats_by_grid.py <run_kernel_trace.csv> <out.csv> [name substring ...]

Output rows: kernel name, grid size (x, threads), workgroup size, calls, total / average / min / max /
median duration in ns, sorted by total time."""
import collections
import csv
import statistics
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    subs = sys.argv[3:]
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        key = (name, int(r["Grid_Size_X"]), int(r.get("Workgroup_Size_X", 0) or 0))
        by[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (name, grid, wg), d in by.items():
        rows.append({"Name": name, "Grid_Size_X": grid, "Workgroup_Size_X": wg, "Calls": len(d),
                     "TotalDurationNs": sum(d), "AverageNs": round(statistics.mean(d), 1),
                     "MedianNs": statistics.median(d), "MinNs": min(d), "MaxNs": max(d)})
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:25]:
        print(f"{r['TotalDurationNs'] / 1e6:10.2f} ms {r['Calls']:6d} x {r['AverageNs'] / 1e3:9.2f} us  grid {r['Grid_Size_X']:8d}  "
              f"{r['Name'][:110]}")


if __name__ == "__main__":
    main()
