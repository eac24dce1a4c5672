#!/usr/bin/env python3
"""Summary of tools/gpu_x6pmc_shapes.sh: per x6 shape at ROWS rows, the kernel's average duration
(kernel-trace stats), fp32-equivalent TF and its fraction of the x6 peak (2.5 PF dense bf16 / 6), the
algorithmic bytes against the measured HBM traffic (2 x FETCH_SIZE + WRITE_SIZE, KiB counters, FETCH_SIZE
doubled on gfx950: MI355X_MICROARCH.md §HBM), MFMA busy, the effective clock and the stall mix.

    python tools/x6_shapes_summary.py <gpurun_out> <dir prefix> [rows]"""
import collections
import csv
import glob
import json
import os
import sys


def counters(d):
    m = collections.defaultdict(list)
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        return {}
    for r in csv.DictReader(open(f)):
        if "gemm_x6_kernel" in r["Kernel_Name"]:
            m[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in m.items()}


def main():
    root, prefix = sys.argv[1], sys.argv[2]
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 2097152
    out = {}
    for d in sorted(glob.glob(os.path.join(root, prefix + "*"))):
        if not os.path.isdir(d):
            continue
        mode, k, n = os.path.basename(d)[len(prefix):].split("_")
        k, n = int(k), int(n)
        st = [r for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv")))
              if "gemm_x6_kernel" in r["Name"]]
        if not st:
            continue
        ns = float(st[0]["AverageNs"])
        flop = 2.0 * rows * k * n
        if mode == "bwd":  # grad_next (rows, k) in, y (rows, n) in, grad (rows, n) out
            algo = 4.0 * rows * (k + 2 * n)
            shape = f"backward {n}<-{k}"
        elif mode == "fwd":  # x (rows, k) in, y (rows, n) out
            algo = 4.0 * rows * (k + n)
            shape = f"forward {k}->{n}"
        elif mode == "loss":  # x (rows, k) + action (2) / logprob / advantage per row in, gz (rows, n) out
            algo = 4.0 * rows * (k + n + 4)
            shape = f"last layer + loss {k}->{n}"
        else:  # grad (rows, n) and x (rows, k) in; the (splits, n, k) partials out are not counted
            algo = 4.0 * rows * (k + n)
            shape = f"weight gradient {n}x{k}"
        c = {}
        for p in ("p1", "p2", "p3", "p4"):
            c.update(counters(os.path.join(d, p)))
        r = {"kernel": st[0]["Name"], "avg_ms": ns / 1e6, "calls": int(st[0]["Calls"]),
             "tflops_fp32_equiv": flop / ns / 1e3, "frac_x6_peak": flop / ns / 1e3 / (2500.0 / 6),
             "algorithmic_bytes": algo, "algorithmic_GBps": algo / ns}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            traffic = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            r.update(hbm_bytes=traffic, traffic_over_algorithmic=traffic / algo, fetch_x2_bytes=2 * c["FETCH_SIZE"] * 1024,
                     write_bytes=c["WRITE_SIZE"] * 1024)
        if "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
            r["clock_ghz"] = cyc / ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                r["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            r["valu_insts_per_mfma"] = c.get("SQ_INSTS_VALU", 0) / max(1.0, c.get("SQ_INSTS_MFMA", 1))
        if "SQ_WAVE_CYCLES" in c:
            for k2 in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                       "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if k2 in c:
                    r[k2.lower() + "_frac"] = c[k2] / c["SQ_WAVE_CYCLES"]
        r["counters"] = c
        out[shape] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
