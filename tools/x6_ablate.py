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
  biasinit  (correct results, other rounding) the forward's accumulators start at the bias instead of
            zero (no bias add in the epilogue)
  fasttanh  (less accurate: timing only) tanh as 2 / (1 + exp(-2z)) - 1
  onewave   (correct results) the forward / backward's 256 x 128 block as 4 waves of 64 x 128 (one wave per
            SIMD, 512 registers) instead of 8 of 64 x 64
  fwdnt     (correct results) the forward's epilogue stores nontemporal, as the backward's
  stcontig  (timing only) every epilogue store instruction writes 1 KB of contiguous memory
  ldcontig  (timing only) every backward epilogue y load (but the prefetched group) reads 1 KB contiguous
  nostore   the forward / backward epilogues compute everything but store only under a never-true guard
  nobar     the K loop's two barriers per K-tile pair removed (races: timing only)
  iouter    (correct results) the k-step's MFMAs i-tile-outer: the Q fragments held, the P fragments of
            one i tile at a time (72 instead of 96 fragment registers)
  ypreN     (correct results) the backward requests N of its 4 y row groups during the item's last
            K-tile pair (1 in the product)
  (a start delay of the forward / backward row bands' blocks in 2, 4 or 8 phases over one work item, so
  that their epilogues do not reach HBM at once, changed nothing and was not kept:
  profiles/r04_gemm_x6_stagger_iouter_not_kept.log; nor did a ring of four register-staged K tiles in
  flight instead of two, profiles/r04_gemm_x6_depth4_ring_not_kept.log)
Earlier ablations (nopstage, wab; profiles/r03k_*, r03p_*) ran on earlier versions of the
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
    "iouter": [('    u32x4 pf[3][TI], qf[3][TJ];\n    const char* pk = lds + buf * C::BUF;                    // ST_KROW images: plane 0 of P\n    const char* qk = lds + buf * C::BUF + Img<BI>::BYTES;  // and of Q\n#pragma unroll\n    for (int pl = 0; pl < 3; ++pl) {\n#pragma unroll\n      for (int i = 0; i < TI; ++i) {\n        if constexpr (SP == ST_KROW) {\n          const int i0 = wi * C::WTI + 16 * i;\n          pf[pl][i] = tr_frag(pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 0), pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 1));\n        } else {\n          pf[pl][i] = *reinterpret_cast<const u32x4*>(pb + pl * Img<BI>::PS + i * 256);\n        }\n      }\n#pragma unroll\n      for (int j = 0; j < TJ; ++j) {\n        if constexpr (SQ == ST_KROW) {\n          const int j0 = wj * C::WTJ + 16 * j;\n          qf[pl][j] = tr_frag(qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 0), qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 1));\n        } else {\n          qf[pl][j] = *reinterpret_cast<const u32x4*>(qb + pl * Img<BJ>::PS + j * 256);\n        }\n      }\n    }\n    if constexpr (PDMA) {\n      __builtin_amdgcn_sched_barrier(0);\n      between();\n      __builtin_amdgcn_sched_barrier(0);\n    }\n    // the six products, smallest first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi\n    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};\n    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};\n#pragma unroll\n    for (int x = 0; x < 6; ++x)\n#pragma unroll\n      for (int i = 0; i < TI; ++i)\n#pragma unroll\n        for (int j = 0; j < TJ; ++j)\n          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pf[PP[x]][i]),\n                                                              __builtin_bit_cast(bf16x8, qf[QP[x]][j]), acc[i][j], 0, 0, 0);\n', '    u32x4 qf[3][TJ];\n    const char* pk = lds + buf * C::BUF;                    // ST_KROW images: plane 0 of P\n    const char* qk = lds + buf * C::BUF + Img<BI>::BYTES;  // and of Q\n    auto read_p = [&](int pl, int i) -> u32x4 {\n      if constexpr (SP == ST_KROW) {\n        const int i0 = wi * C::WTI + 16 * i;\n        return tr_frag(pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 0), pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 1));\n      } else {\n        return *reinterpret_cast<const u32x4*>(pb + pl * Img<BI>::PS + i * 256);\n      }\n    };\n#pragma unroll\n    for (int pl = 0; pl < 3; ++pl) {\n#pragma unroll\n      for (int j = 0; j < TJ; ++j) {\n        if constexpr (SQ == ST_KROW) {\n          const int j0 = wj * C::WTJ + 16 * j;\n          qf[pl][j] = tr_frag(qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 0), qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 1));\n        } else {\n          qf[pl][j] = *reinterpret_cast<const u32x4*>(qb + pl * Img<BJ>::PS + j * 256);\n        }\n      }\n    }\n    u32x4 pc[3], pn[3];\n#pragma unroll\n    for (int pl = 0; pl < 3; ++pl) pc[pl] = read_p(pl, 0);\n    // the six products, smallest first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi (per accumulator\n    // the same order as product-outer: the same bits)\n    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};\n    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};\n#pragma unroll\n    for (int i = 0; i < TI; ++i) {\n      if (i + 1 < TI) {\n#pragma unroll\n        for (int pl = 0; pl < 3; ++pl) pn[pl] = read_p(pl, i + 1);\n      }\n      if constexpr (PDMA) {\n        if (i == TI - 1) {\n          __builtin_amdgcn_sched_barrier(0);\n          between();\n          __builtin_amdgcn_sched_barrier(0);\n        }\n      }\n#pragma unroll\n      for (int x = 0; x < 6; ++x)\n#pragma unroll\n        for (int j = 0; j < TJ; ++j)\n          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pc[PP[x]]),\n                                                              __builtin_bit_cast(bf16x8, qf[QP[x]][j]), acc[i][j], 0, 0, 0);\n#pragma unroll\n      for (int pl = 0; pl < 3; ++pl) pc[pl] = pn[pl];\n    }\n')],
    "ypre2": [("constexpr int kYPre = 1;", "constexpr int kYPre = 2;")],
    "ypre4": [("constexpr int kYPre = 1;", "constexpr int kYPre = 4;")],
    "nostore": [("          *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;\n          if constexpr (EPI == EPI_TANH_OUT) {",
                 "          if (v[0] == 1234.5f) *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;\n          if constexpr (EPI == EPI_TANH_OUT) {"),
                ("          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));",
                 "          if (v[0] == 1234.5f) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));")],
    "biasinit": [("      for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};",
                  "      for (int j = 0; j < TJ; ++j) {\n"
                  "        if constexpr (EPI == EPI_TANH || EPI == EPI_TANH_OUT) {\n"
                  "          const int il0 = wi * C::WTI + 16 * i + 4 * fg;\n"
                  "          acc[i][j] = (f32x4){epi_lds[il0], epi_lds[il0 + 1], epi_lds[il0 + 2], epi_lds[il0 + 3]};\n"
                  "        } else {\n"
                  "          acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};\n"
                  "        }\n"
                  "      }"),
                 ("for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + epi_lds[il + r]);", "for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r]);")],
    "fasttanh": [("for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + epi_lds[il + r]);",
                  "for (int r = 0; r < 4; ++r) v[r] = fmaf(2.0f, __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.8853900817779268f * (v[r] + epi_lds[il + r]))), -1.0f);")],
    # timing only: each epilogue store / y load instruction on 1 KB of contiguous memory (the same bytes
    # per item, other addresses) instead of 16 rows x 64 B
    "stcontig": [("          *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;",
                  "          *reinterpret_cast<f32x4*>(a.out + (((int64_t)(it * a.nj + jt) * (C::THREADS / 64) + wv) * (TI * TJ) + i * TJ + j) * 256 + lane * 4) = v;"),
                 ("          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));",
                  "          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + (((int64_t)(it * a.nj + jt) * (C::THREADS / 64) + wv) * (TI * TJ) + i * TJ + j) * 256 + lane * 4));")],
    "ldcontig": [("yrest[j][i] = *reinterpret_cast<const f32x4*>(a.y + ((int64_t)jb + 16 * j + fr) * a.ldo + ib + 16 * i + 4 * fg);",
                  "yrest[j][i] = *reinterpret_cast<const f32x4*>(a.y + (((int64_t)(it * a.nj + jt) * (C::THREADS / 64) + wv) * (TI * TJ) + i * TJ + j) * 256 + lane * 4);")],
    "fwdnt": [("          *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;",
               "          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig));")],
    "onewave": [("using CfgB = Cfg<256, 128, 4, 2>;", "using CfgB = Cfg<256, 128, 4, 1>;")],
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
