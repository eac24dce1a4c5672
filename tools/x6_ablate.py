#!/usr/bin/env python3
"""Profiling-only: builds ablated copies of csrc/vss_gemm_x6.hip into tools/_build/libx6_<name>.so
(WRONG RESULTS -- timing only) to locate the K loop's non-MFMA time:
  nosplit   the staging writes store the raw fp32 words as planes (no split VALU)
  nobar     no workgroup barrier in the K loop (races: timing only)
  noglobal  the K loop issues no global loads (the staged registers are re-written as they are)
  qsmall    every item reads the Q rows of j tile 0 (L2-resident activations)
Usage: python tools/x6_ablate.py nosplit nobar noglobal nosplit+noglobal"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_gemm_x6.hip")
PATCH = {
    "nosplit": [("      split8(v, hi, mid, lo);", "      hi = src[u][0]; mid = src[u][1]; lo = src[u][0]; (void)v;")],
    "nobar": [("""      mfma_tile(0);
      swrite(r1, 1);
      __syncthreads();""", """      mfma_tile(0);
      swrite(r1, 1);
      __builtin_amdgcn_sched_barrier(0);"""),
              ("""      mfma_tile(1);
      swrite(r0, 0);
      __syncthreads();""", """      mfma_tile(1);
      swrite(r0, 0);
      __builtin_amdgcn_sched_barrier(0);""")],
    "qsmall": [("""    else fq = reinterpret_cast<const char*>(a.q) + (int64_t)jt * BJ * a.ldq * 4;""",
                """    else fq = reinterpret_cast<const char*>(a.q) + (int64_t)(jt & 0) * BJ * a.ldq * 4;""")],
    "noglobal": [("""      gload(r1);
      mfma_tile(1);""", """      mfma_tile(1);"""), ("""      gload(r0);
    }""", """    }""")],
}


def main():
    os.makedirs(os.path.join(REPO, "tools", "_build"), exist_ok=True)
    for name in sys.argv[1:]:
        s = open(SRC).read()
        for part in name.split("+"):
            for old, new in PATCH[part]:
                assert old in s, (part, old)
                s = s.replace(old, new)
        tag = name.replace("+", "_")
        path = os.path.join(REPO, "tools", "_build", f"x6_{tag}.hip")
        open(path, "w").write(s)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                        "-o", os.path.join(REPO, "tools", "_build", f"libx6_{tag}.so"), path], check=True)
        print("built", tag)


if __name__ == "__main__":
    main()
