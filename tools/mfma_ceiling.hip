// Profiling-only: the MFMA ceiling the x6 GEMMs (csrc/vss_gemm_x6.hip) run against, on random data.
//
// Each wave runs the x6 kernels' inner-loop MFMA mix with no global memory in the loop: per step 6 x
// 4 x 4 v_mfma_f32_16x16x32_bf16 (six products of a 64 x 64 wave tile, K = 32) into 16 accumulators.
//   regs: the operand fragments stay in registers (the bare matrix-core rate at the clock the chip
//         holds for this instruction stream)
//   lds:  the 24 fragments are re-read from an LDS image every step, as the GEMMs' k-steps read theirs
// 256 workgroups x 8 waves (2 per SIMD, the GEMMs' occupancy), launched back to back for >= 2 s; the
// in-kernel clock is s_memtime / s_memrealtime (100 MHz) stamped around the loop by each wave's lane 0
// into a buffer of its own (MI355X_MICROARCH.md, DVFS give-back item 6).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/_build/mfma_ceiling tools/mfma_ceiling.hip
//   tools/_build/mfma_ceiling            -> one JSON line per variant
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int TI = 4, TJ = 4, THREADS = 512, GRID = 256;

template <bool LDS>
__global__ __launch_bounds__(THREADS, 1) void ceiling_kernel(const u32x4* __restrict__ src, int steps, float* out,
                                                             uint64_t* stamps) {
  __shared__ u32x4 img[24 * 64 * 4];  // 24 fragments x 64 lanes, x4 so waves read different slots
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u32x4 pf[3][TI], qf[3][TJ];
  for (int pl = 0; pl < 3; ++pl) {
    for (int i = 0; i < TI; ++i) pf[pl][i] = src[((pl * TI + i) * 64 + lane) + blockIdx.x % 7];
    for (int j = 0; j < TJ; ++j) qf[pl][j] = src[((12 + pl * TJ + j) * 64 + lane) + blockIdx.x % 5];
  }
  if (LDS) {
    for (int f = threadIdx.x; f < 24 * 64 * 4; f += THREADS) img[f] = src[f % (24 * 64)];
    __syncthreads();
  }
  f32x4 acc[TI][TJ];
  for (int i = 0; i < TI; ++i)
    for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int slot = (wv & 3) * 24 * 64;
  for (int s = 0; s < steps; ++s) {
    if (LDS) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < TI; ++i) pf[pl][i] = img[slot + (pl * TI + i) * 64 + lane];
#pragma unroll
        for (int j = 0; j < TJ; ++j) qf[pl][j] = img[slot + (12 + pl * TJ + j) * 64 + lane];
      }
    }
    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
    for (int x = 0; x < 6; ++x)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pf[PP[x]][i]),
                                                              __builtin_bit_cast(bf16x8, qf[QP[x]][j]), acc[i][j], 0,
                                                              0, 0);
    if (LDS) __syncthreads();  // the GEMMs' per-k-step barrier
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
  for (int i = 0; i < TI; ++i)
    for (int j = 0; j < TJ; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * THREADS + threadIdx.x] = sum;
  if (lane == 0) {
    const int w = blockIdx.x * (THREADS / 64) + wv;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                   \
    }                                                             \
  } while (0)

template <bool LDS>
static int run(const char* name, const u32x4* src, float* out, uint64_t* stamps, int steps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // warm up (clock settles under load) then time back-to-back launches for >= 2 s
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(ceiling_kernel<LDS>, dim3(GRID), dim3(THREADS), 0, 0, src, steps, out, stamps);
  CK(hipDeviceSynchronize());
  int launches = 0;
  float ms = 0.f;
  CK(hipEventRecord(e0, 0));
  while (ms < 2000.f) {
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(ceiling_kernel<LDS>, dim3(GRID), dim3(THREADS), 0, 0, src, steps, out, stamps);
    launches += 10;
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  const int waves = GRID * THREADS / 64;
  std::vector<uint64_t> st(2 * waves);
  CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> clk(waves);
  for (int w = 0; w < waves; ++w) clk[w] = (double)st[2 * w] / (double)st[2 * w + 1] * 100e6;
  std::sort(clk.begin(), clk.end());
  const double mfma = (double)launches * waves * steps * 6 * TI * TJ;
  const double tf = mfma * 2 * 16 * 16 * 32 / (ms * 1e-3) / 1e12;
  printf("{\"variant\": \"%s\", \"launches\": %d, \"ms\": %.1f, \"bf16_tflops\": %.1f, \"fp32_equivalent_x6_tflops\": %.1f, "
         "\"frac_of_2500\": %.4f, \"in_kernel_clock_ghz_median\": %.3f, \"clock_min\": %.3f, \"clock_max\": %.3f}\n",
         name, launches, ms, tf, tf / 6, tf / 2500.0, clk[waves / 2] / 1e9, clk[0] / 1e9, clk[waves - 1] / 1e9);
  return 0;
}

int main() {
  const size_t n = 24 * 64 + 16;
  std::vector<uint32_t> h(4 * n);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& v : h) {  // random bf16 pairs with exponents near 1 (as the split planes' hi parts)
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    const uint32_t a = 0x3F00u | (uint32_t)(x & 0x80FF), b = 0x3F00u | (uint32_t)((x >> 16) & 0x80FF);
    v = a | (b << 16);
  }
  u32x4* src;
  float* out;
  uint64_t* stamps;
  CK(hipMalloc(&src, h.size() * 4));
  CK(hipMalloc(&out, GRID * THREADS * 4));
  CK(hipMalloc(&stamps, GRID * THREADS / 64 * 16));
  CK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  if (run<false>("regs", src, out, stamps, 2000)) return 1;
  if (run<true>("lds", src, out, stamps, 2000)) return 1;
  CK(hipFree(src));
  CK(hipFree(out));
  CK(hipFree(stamps));
  return 0;
}
