#!/usr/bin/env python3
"""Profiling-only: builds ablated copies of csrc/vss_gemm_x6.hip into tools/_build/libx6_<name>.so
(WRONG RESULTS -- timing only) to locate the K loop's non-MFMA time:
  nosplit   the staging writes store the raw fp32 words as planes (no split VALU)
  nobar     no workgroup barrier in the K loop (races: timing only)
  noglobal  the K loop issues no global loads (the staged registers are re-written as they are)
  qsmall    every item reads the Q rows of j tile 0 (L2-resident activations)
  nopstage  the weight operand (P) is staged once per block and never re-loaded or re-written (the
            upper bound of taking P's staging out of the K loop, e.g. by LDS-DMA)
  bigfirst  (correct results) the six products largest first (hi.hi, hi.mid, mid.hi, hi.lo,
            mid.mid, lo.hi): the first MFMAs of a K tile need only the hi planes' fragments
  notanh    the forward epilogue adds the bias but skips the tanh (its VALU cost)
  noy       the backward epilogue reuses the prefetched first y row group for every row group
            (the cost of the epilogue's y loads)
  wab       (correct results) the staging write placed AFTER the barrier: per K tile,
            swrite(next) -> gload(next + 2) -> MFMAs -> barrier (guide T14 / G15)
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
    "nopstage": [("""    load_op<SP, BI, PI, C>(s.v, fp, a.ldp, k0, a.pps);
    load_op<SQ, BJ, PJ, C>(s.v + PI, fq, a.ldq, k0, 0);""", """    if (f_item == slot && f_kt == 0) load_op<SP, BI, PI, C>(s.v, fp, a.ldp, k0, a.pps);
    load_op<SQ, BJ, PJ, C>(s.v + PI, fq, a.ldq, k0, 0);"""),
                 ("""    write_op<SP, BI, PI, C>(s.v, base);
    write_op<SQ, BJ, PJ, C>(s.v + PI, base + Img<BI>::BYTES);""", """    if (buf == 0 && first_write) write_op<SP, BI, PI, C>(s.v, base);
    if (buf == 1 && first_write1) write_op<SP, BI, PI, C>(s.v, base);
    write_op<SQ, BJ, PJ, C>(s.v + PI, base + Img<BI>::BYTES);
    if (buf == 0) first_write = false; else first_write1 = false;"""),
                 ("""  auto swrite = [&](const Stage<C>& s, int buf) {""", """  bool first_write = true, first_write1 = true;
  auto swrite = [&](const Stage<C>& s, int buf) {""")],
    "bigfirst": [("""    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};""", """    constexpr int PP[6] = {0, 0, 1, 0, 1, 2};
    constexpr int QP[6] = {0, 1, 0, 2, 1, 0};""")],
    "wab": [("""      mfma_tile(0);
      swrite(r1, 1);
      __syncthreads();
      gload(r1);
      mfma_tile(1);
      swrite(r0, 0);
      __syncthreads();
      gload(r0);""", """      swrite(r1, 1);
      gload(r1);
      mfma_tile(0);
      __syncthreads();
      swrite(r0, 0);
      gload(r0);
      mfma_tile(1);
      __syncthreads();"""), ("""  gload(r0);  // K tile 0
  swrite(r0, 0);
  gload(r1);  // K tile 1
  gload(r0);  // K tile 2
  __syncthreads();""", """  gload(r0);  // K tile 0
  swrite(r0, 0);
  gload(r1);  // K tile 1
  gload(r0);  // K tile 2
  __syncthreads();""")],
    "notanh": [("v[r] = tanh_f32(v[r] + epi_lds[il + r]);", "v[r] = v[r] + epi_lds[il + r];")],
    "noy": [("const f32x4 yv = j == 0 ? ypre[i] : *reinterpret_cast<const f32x4*>(a.y + jg * a.ldo + ig);",
             "const f32x4 yv = ypre[i];")],
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
