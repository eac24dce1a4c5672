#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/policy_bench.py (tools/gpu_check.sh step `pol`) for
the rollout policy kernel: MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
1,024 SIMDs) (MI355X_MICROARCH.md; 32 busy cycles per v_mfma_f32_16x16x4_f32), and the wave-cycle
split of the SQ pass (quad-cycles: WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY = issue
stalls incl. the busy MFMA pipe, ACTIVE_INST_ANY = issuing).

    python tools/policy_pmc.py --tag r03d [--out profiles/r03d_pmc_policy.json]
"""
import argparse
import collections
import csv
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def means(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if "policy_kernel" in r["Kernel_Name"]:
            d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    g = os.path.join(REPO, "gpurun_out")
    res = {}
    for sub in (f"pmc_policy_{a.tag}", f"pmc_policy_sq_{a.tag}"):
        p = os.path.join(g, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            for k, m in means(p).items():
                res.setdefault(k, {}).update(m)
    for k, m in res.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            m["kernel_cycles_per_xcd"] = m["GRBM_GUI_ACTIVE"] / 8
            m["mfma_utilization"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["kernel_cycles_per_xcd"] * 1024)
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
    out = a.out or os.path.join(REPO, "profiles", f"{a.tag}_pmc_policy.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, m in res.items():
        print(k[:45], {c: round(v, 3) for c, v in m.items() if c.endswith("frac") or c == "mfma_utilization"})


if __name__ == "__main__":
    main()
