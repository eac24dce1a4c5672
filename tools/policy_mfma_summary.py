#!/usr/bin/env python3
"""Summarise the policy kernel's MFMA utilisation from a rocprofv3 --pmc pass
(tools/gpu_check.sh step `profall`: SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA
SQ_WAVES SQ_BUSY_CYCLES over tools/policy_bench.py) into profiles/<tag>_pmc_policy_mfma.json.

utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs): the matrix-core
busy cycles summed over all SIMDs over the SIMD-cycles the kernel was active."""
import argparse
import collections
import csv
import json
import os
import shutil
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    args = ap.parse_args()
    src = os.path.join(REPO, "gpurun_out", f"pmc_policy_{args.tag}", "run_counter_collection.csv")
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(src)):
        if "policy_kernel" in r["Kernel_Name"]:
            by[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in by.items():
        m = {n: statistics.mean(v) for n, v in c.items()}
        m["kernel_cycles_per_xcd"] = m["GRBM_GUI_ACTIVE"] / 8
        m["mfma_utilization"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["kernel_cycles_per_xcd"] * 1024)
        m["note"] = ("SQ_VALU_MFMA_BUSY_CYCLES = 32 cycles x SQ_INSTS_MFMA (v_mfma_f32_16x16x4_f32); "
                     "GRBM_GUI_ACTIVE is the sum over 8 XCDs; 1024 SIMDs")
        out[k] = m
    dst = os.path.join(REPO, "profiles")
    shutil.copy(src, os.path.join(dst, f"{args.tag}_pmc_policy.csv"))
    with open(os.path.join(dst, f"{args.tag}_pmc_policy_mfma.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: round(v["mfma_utilization"], 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
