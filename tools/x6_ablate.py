#!/usr/bin/env python3
"""Profiling-only: builds ablated copies of csrc/vss_gemm_x6.hip into tools/_build/libx6_<name>.so
(WRONG RESULTS -- timing only, except bigfirst) to locate a kernel's non-MFMA time; A/B them with
tools/gemm_x6_variants.py:
  nosplit   the activations' staging writes store the raw fp32 words as planes (no split VALU)
  noglobal  the K loop issues no activation loads (the staged registers are written again as they are)
  qsmall    every item reads the Q rows of j tile 0 (L2-resident activations)
  l2k       every K loop cycles over its first 4 K tiles (the staged operands L2-resident)
  bigfirst  (correct results) the six products largest first
  notanh    the forward epilogue adds the bias but skips the tanh (its VALU cost)
  noy       the backward epilogue reuses the prefetched first y row group for every row group
            (the cost of the epilogue's y loads)
  noepi     the forward / backward epilogues neither transform nor store (a never-true guard keeps
            the accumulators live): the K loop's time alone
  nobar     the K loop's two barriers per K-tile pair removed (races: timing only)
Earlier ablations (nobar, nopstage, wab; profiles/r03k_*, r03p_*) ran on earlier versions of the
kernel and were retired with the code they patched.
Usage: python tools/x6_ablate.py nosplit noglobal nosplit+noglobal"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_gemm_x6.hip")
PATCH = {
    # the activations' staging writes store raw fp32 words as planes (no split VALU)
    "nosplit": [("    split8(v, hi, mid, lo);\n    char* d", "    hi = src[u][0]; mid = src[u][1]; lo = src[u][0]; (void)v;\n    char* d")],
    "qsmall": [("""    else fq = reinterpret_cast<const char*>(a.q) + (int64_t)jt * BJ * a.ldq * 4;""",
                """    else fq = reinterpret_cast<const char*>(a.q) + (int64_t)(jt & 0) * BJ * a.ldq * 4;""")],
    "bigfirst": [("""    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};""", """    constexpr int PP[6] = {0, 0, 1, 0, 1, 2};
    constexpr int QP[6] = {0, 1, 0, 2, 1, 0};""")],
    "l2k": [("const int64_t k0 = fk0 + (int64_t)f_kt * KT;", "const int64_t k0 = fk0 + (int64_t)(f_kt & 3) * KT;")],
    "notanh": [("v[r] = tanh_f32(v[r] + epi_lds[il + r]);", "v[r] = v[r] + epi_lds[il + r];")],
    "noy": [("yrest[j][i] = *reinterpret_cast<const f32x4*>(a.y + ((int64_t)jb + 16 * j + fr) * a.ldo + ib + 16 * i + 4 * fg);",
             "yrest[j][i] = ypre[0][i];")],
    "noepi": [("          for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + epi_lds[il + r]);\n          *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;",
               "          for (int r = 0; r < 1; ++r) (void)r;\n          if (v[0] == 1234.5f) *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;"),
              ("          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));",
               "          if (v[0] == 1234.5f) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));"),
              ("            v[r] = v[r] * fmaf(-yv[r], yv[r], 1.0f);\n            cs[i][r] += v[r];", "            (void)yv;"),
              ("yrest[j][i] = *reinterpret_cast<const f32x4*>(a.y + ((int64_t)jb + 16 * j + fr) * a.ldo + ib + 16 * i + 4 * fg);",
               "yrest[j][i] = ypre[0][i];")],
    "nobar": [("      swrite(r1, 1);\n      __syncthreads();", "      swrite(r1, 1);"),
              ("      swrite(r0, 0);\n      __syncthreads();", "      swrite(r0, 0);")],
    # the K loop issues no global loads (the staged registers are written again as they are)
    "noglobal": [("      gload(r1);\n", ""), ("      gload(r0);\n", "")],
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
