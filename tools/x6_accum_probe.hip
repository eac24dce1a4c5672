// Profiling-only (numerics): where the x6 GEMMs' column-correlated error comes from (tools/x6_bias_probe.py: the
// column sums of a 524,288-row x6 product are 30 x further from fp64 than torch's fp32 ones, while each
// element's error is an fp32 GEMM's and bf16-exact inputs show none of it).  One wave per 16 x 16 output tile,
// operands read from global memory and split exactly into hi / mid / lo bf16 planes as csrc/vss_gemm_x6.hip
// does, v_mfma_f32_16x16x32_bf16 per K step of 32, with the accumulation variants:
//   0 product order of the kernel (lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi) into one accumulator
//   1 the same six products, largest first
//   2 three accumulators (hi.hi | mid.hi + hi.mid | lo.hi + hi.lo + mid.mid), added at the end in fp32
//   3 a fresh accumulator per K step (the six products), added to the running sum in fp32 (RNE)
//   4 the split without the lo plane's products (hi.hi, mid.hi, hi.mid, mid.mid)
//   5 the five smaller products of a K step into a fresh accumulator, added to the running sum in fp32,
//     then hi.hi into the running sum (one temporary per output tile)
//   6 two accumulators: hi.hi | the five smaller products, added at the end
//   7 the five smaller products into the running sum, hi.hi into a zero accumulator added in fp32 per K step
// and reports, against an fp64 GEMM of the same inputs: offset = mean(e) / rms(e), colsum = relative error of
// the column sums, elem = relative Frobenius error.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/x6_accum_probe tools/x6_accum_probe.hip && /tmp/x6_accum_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static int M = 65536, N = 256, K = 256;  // PROBE_M / PROBE_N / PROBE_K override

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ void split8(const float (&v)[8], u32x4& hi, u32x4& mid, u32x4& lo) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    const uint32_t h = pk_bf16(a, b);
    const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xFFFF0000u);
    const uint32_t m = pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(m << 16), sb = rb - __uint_as_float(m & 0xFFFF0000u);
    hi[p] = h;
    mid[p] = m;
    lo[p] = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
  }
}
__device__ __forceinline__ f32x4 mf(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// C[m][n] = sum_k A[m][k] B[n][k]  (both K-contiguous); one wave per 16 x 16 tile
template <int V>
__global__ __launch_bounds__(64) void x6_tile(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C,
                                              int M, int N, int K) {
  const int l = threadIdx.x, tm = blockIdx.x, tn = blockIdx.y;
  const int r = l & 15, g = l >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, a2 = acc, a3 = acc;
  for (int k0 = 0; k0 < K; k0 += 32) {
    float av[8], bv[8];
    for (int e = 0; e < 8; ++e) {
      av[e] = A[(int64_t)(tm * 16 + r) * K + k0 + 8 * g + e];
      bv[e] = B[(int64_t)(tn * 16 + r) * K + k0 + 8 * g + e];
    }
    u32x4 ah, am, al, bh, bm, bl;
    split8(av, ah, am, al);
    split8(bv, bh, bm, bl);
    if constexpr (V == 0) {
      acc = mf(al, bh, acc); acc = mf(ah, bl, acc); acc = mf(am, bm, acc);
      acc = mf(am, bh, acc); acc = mf(ah, bm, acc); acc = mf(ah, bh, acc);
    } else if constexpr (V == 1) {
      acc = mf(ah, bh, acc); acc = mf(ah, bm, acc); acc = mf(am, bh, acc);
      acc = mf(am, bm, acc); acc = mf(ah, bl, acc); acc = mf(al, bh, acc);
    } else if constexpr (V == 2) {
      a3 = mf(al, bh, a3); a3 = mf(ah, bl, a3); a3 = mf(am, bm, a3);
      a2 = mf(am, bh, a2); a2 = mf(ah, bm, a2);
      acc = mf(ah, bh, acc);
    } else if constexpr (V == 3) {
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
      t = mf(al, bh, t); t = mf(ah, bl, t); t = mf(am, bm, t);
      t = mf(am, bh, t); t = mf(ah, bm, t); t = mf(ah, bh, t);
      for (int i = 0; i < 4; ++i) acc[i] += t[i];
    } else if constexpr (V == 4) {
      acc = mf(am, bm, acc); acc = mf(am, bh, acc); acc = mf(ah, bm, acc); acc = mf(ah, bh, acc);
    } else if constexpr (V == 5) {
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
      t = mf(al, bh, t); t = mf(ah, bl, t); t = mf(am, bm, t); t = mf(am, bh, t); t = mf(ah, bm, t);
      for (int i = 0; i < 4; ++i) acc[i] += t[i];
      acc = mf(ah, bh, acc);
    } else if constexpr (V == 7) {
      acc = mf(al, bh, acc); acc = mf(ah, bl, acc); acc = mf(am, bm, acc); acc = mf(am, bh, acc); acc = mf(ah, bm, acc);
      const f32x4 t = mf(ah, bh, (f32x4){0.f, 0.f, 0.f, 0.f});
      for (int i = 0; i < 4; ++i) acc[i] += t[i];
    } else {
      a2 = mf(al, bh, a2); a2 = mf(ah, bl, a2); a2 = mf(am, bm, a2); a2 = mf(am, bh, a2); a2 = mf(ah, bm, a2);
      acc = mf(ah, bh, acc);
    }
  }
  if constexpr (V == 2)
    for (int i = 0; i < 4; ++i) acc[i] = acc[i] + (a2[i] + a3[i]);
  if constexpr (V == 6)
    for (int i = 0; i < 4; ++i) acc[i] = acc[i] + a2[i];
  // accumulator lane l: rows 4 g .. + 3 (of A's 16), column r (of B's 16)
  for (int i = 0; i < 4; ++i) C[(int64_t)(tm * 16 + 4 * g + i) * N + tn * 16 + r] = acc[i];
}

__global__ void ref64(const float* __restrict__ A, const float* __restrict__ B, double* __restrict__ C, int M, int N, int K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)M * N) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += (double)A[(int64_t)m * K + k] * (double)B[(int64_t)n * K + k];
  C[idx] = s;
}

static double normal(uint64_t& s) {  // Box-Muller on xorshift
  auto u = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return ((s >> 11) + 0.5) * (1.0 / 9007199254740992.0);
  };
  return sqrt(-2.0 * log(u())) * cos(6.283185307179586 * u());
}

template <int V>
static void run(const char* name, const float* dA, const float* dB, float* dC, const std::vector<double>& ref) {
  hipLaunchKernelGGL(x6_tile<V>, dim3(M / 16, N / 16), dim3(64), 0, 0, dA, dB, dC, M, N, K);
  std::vector<float> c((size_t)M * N);
  (void)hipMemcpy(c.data(), dC, c.size() * 4, hipMemcpyDeviceToHost);
  double se = 0, se2 = 0, sr2 = 0, cs2 = 0, csr2 = 0;
  std::vector<double> cs(N, 0.0), csr(N, 0.0);
  for (size_t i = 0; i < c.size(); ++i) {
    const double e = (double)c[i] - ref[i];
    se += e;
    se2 += e * e;
    sr2 += ref[i] * ref[i];
    cs[i % N] += c[i];
    csr[i % N] += ref[i];
  }
  for (int n = 0; n < N; ++n) {
    cs2 += (cs[n] - csr[n]) * (cs[n] - csr[n]);
    csr2 += csr[n] * csr[n];
  }
  const double cnt = (double)c.size();
  printf("{\"variant\": \"%s\", \"offset\": %.4f, \"colsum\": %.3e, \"elem\": %.3e}\n", name, (se / cnt) / sqrt(se2 / cnt),
         sqrt(cs2 / csr2), sqrt(se2 / sr2));
  fflush(stdout);
}

int main() {
  if (getenv("PROBE_M")) M = atoi(getenv("PROBE_M"));
  if (getenv("PROBE_N")) N = atoi(getenv("PROBE_N"));
  if (getenv("PROBE_K")) K = atoi(getenv("PROBE_K"));
  printf("{\"M\": %d, \"N\": %d, \"K\": %d}\n", M, N, K);
  std::vector<float> a((size_t)M * K), b((size_t)N * K);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& v : a) v = (float)(normal(s) * 1e-3);
  for (auto& v : b) v = (float)(normal(s) / 16.0);
  float *dA, *dB, *dC;
  double* dR;
  (void)hipMalloc(&dA, a.size() * 4);
  (void)hipMalloc(&dB, b.size() * 4);
  (void)hipMalloc(&dC, (size_t)M * N * 4);
  (void)hipMalloc(&dR, (size_t)M * N * 8);
  (void)hipMemcpy(dA, a.data(), a.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(ref64, dim3((M * N + 255) / 256), dim3(256), 0, 0, dA, dB, dR, M, N, K);
  std::vector<double> ref((size_t)M * N);
  (void)hipMemcpy(ref.data(), dR, ref.size() * 8, hipMemcpyDeviceToHost);
  run<0>("0 kernel order, one accumulator", dA, dB, dC, ref);
  run<1>("1 largest first, one accumulator", dA, dB, dC, ref);
  run<2>("2 three accumulators by magnitude", dA, dB, dC, ref);
  run<3>("3 fresh accumulator per K step + fp32 add", dA, dB, dC, ref);
  run<4>("4 without the lo-plane products", dA, dB, dC, ref);
  run<5>("5 smaller products into a fresh accumulator per K step, fp32 add, then hi.hi", dA, dB, dC, ref);
  run<6>("6 two accumulators: hi.hi | the smaller five", dA, dB, dC, ref);
  run<7>("7 smaller five into the running sum, hi.hi into a zero accumulator + fp32 add", dA, dB, dC, ref);
  return 0;
}
