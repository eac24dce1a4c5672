// vss_update.hip — PPO-update helper on gfx950 (ppo_continuous_action_isaacgym.py:306-353).
//
// The update back-propagates through the Agent's tanh MLPs (ppo…:104-125).  For each hidden
// layer torch issues two memory-bound passes over the (rows x cols) gradient: tanh_backward
// (gz = gy * (1 - y^2): read gy, y, write gz) and the bias gradient (db = sum over rows of gz:
// read gz again).  This kernel does both in one pass: every workgroup owns a fixed set of row
// tiles, writes gz and one row of column sums; the caller reduces the (workgroups x cols)
// partial sums (a few MB) to db.  The tile assignment and the order of the sums are fixed, so
// db is deterministic.  HBM bytes per element: 12 (gy, y read, gz write) instead of 16.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"

namespace vupd {

// tuning knobs (tools/tanh_grad_bench.py builds variants; the product uses the defaults)
#ifndef VSS_TG_U
#define VSS_TG_U 8
#endif
#ifndef VSS_TG_WAVES
#define VSS_TG_WAVES 4
#endif
#ifndef VSS_TG_MAXBLK
#define VSS_TG_MAXBLK 2048
#endif
#ifndef VSS_TG_NT
#define VSS_TG_NT 0
#endif
constexpr int kThreads = 256;
constexpr int kU = VSS_TG_U;                   // rows per lane in flight (2 x kU 16-B loads before the first use)
constexpr int64_t kMaxBlocks = VSS_TG_MAXBLK;  // the partial sums are (blocks x cols)

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld(const float4* p) {
#if VSS_TG_NT
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}

__device__ __forceinline__ float4 tanh_grad(float4 g, float4 y) {
  // d tanh(z) / dz = 1 - tanh(z)^2
  return make_float4(g.x * fmaf(-y.x, y.x, 1.0f), g.y * fmaf(-y.y, y.y, 1.0f), g.z * fmaf(-y.z, y.z, 1.0f),
                     g.w * fmaf(-y.w, y.w, 1.0f));
}

__device__ __forceinline__ void add4(float4& a, float4 b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

__host__ __device__ constexpr int64_t tile_rows(int cols) { return (int64_t)kU * (kThreads / (cols / 4)); }

__host__ inline int64_t n_blocks(int64_t rows, int cols) {
  const int64_t tiles = (rows + tile_rows(cols) - 1) / tile_rows(cols);
  return tiles < kMaxBlocks ? tiles : kMaxBlocks;
}

// C4 = cols / 4 float4 columns; RG = kThreads / C4 rows per workgroup step.  A tile is kU x RG
// consecutive rows (32 KB of each operand at 512 columns); workgroup b takes tiles b, b + grid,
// ... so at any moment the grid streams one contiguous region (no two workgroups start at
// addresses that share their low bits, which would pile them onto the same HBM channels).  Lane t
// owns float4 column t % C4 of rows rg, rg + RG, ... of each tile.  Up to 4 waves per SIMD: the
// register budget then holds all 2 kU loads of a lane in flight (at 8 waves the compiler caps it at
// 64 VGPRs and serialises the loads behind the stores).  Measured at 2,097,152 x 512: 5.4 TB/s
// (tools/tanh_grad_bench.py; torch's tanh_backward alone: 6.0 TB/s, + its bias sum: 4.4 TB/s
// effective); a two-register-set software pipeline compiled to a vmcnt(0) per tile and was no
// faster.
template <int C4>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, VSS_TG_WAVES))) void tanh_grad_bias_kernel(
    int64_t rows, const float4* __restrict__ gy, const float4* __restrict__ y, float4* __restrict__ gz,
    float4* __restrict__ partial) {
  constexpr int RG = kThreads / C4;
  constexpr int64_t TILE = (int64_t)kU * RG;
  static_assert(RG * C4 == kThreads, "cols / 4 must divide the workgroup size");
  __shared__ float4 red[kThreads];
  const int t = threadIdx.x, c4 = t % C4, rg = t / C4;
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const int64_t full_tiles = rows / TILE;
  int64_t tile = blockIdx.x;
  for (; tile < full_tiles; tile += gridDim.x) {
    const int64_t base = (tile * TILE + rg) * C4 + c4;
    float4 g[kU], v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      g[u] = ld(gy + base + u * RG * C4);
      v[u] = ld(y + base + u * RG * C4);
    }
    __builtin_amdgcn_sched_barrier(0);  // all 2 kU loads issued before the first store
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const float4 z = tanh_grad(g[u], v[u]);
      gz[base + u * RG * C4] = z;
      add4(acc, z);
    }
  }
  if (tile == full_tiles) {  // the ragged last tile (rows % TILE), one workgroup
    for (int64_t r = full_tiles * TILE + rg; r < rows; r += RG) {
      const int64_t i = r * C4 + c4;
      const float4 z = tanh_grad(gy[i], y[i]);
      gz[i] = z;
      add4(acc, z);
    }
  }
  red[t] = acc;
  __syncthreads();
  if (rg == 0) {
    float4 s = red[c4];
#pragma unroll
    for (int k = 1; k < RG; ++k) add4(s, red[k * C4 + c4]);
    partial[(int64_t)blockIdx.x * C4 + c4] = s;
  }
}

}  // namespace vupd

extern "C" {

static bool tanh_grad_cols_ok(int32_t cols) {
  return cols == 64 || cols == 128 || cols == 256 || cols == 512 || cols == 1024;
}

int64_t vss_tanh_grad_chunks(int64_t rows, int32_t cols) {
  return (rows < 0 || !tanh_grad_cols_ok(cols)) ? -1 : vupd::n_blocks(rows, cols);
}

int vss_tanh_grad_bias(void* stream, int64_t rows, int32_t cols, const float* grad_out, const float* y,
                       float* grad_in, float* bias_partial) {
  auto bad = [](const void* p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) != 0; };
  if (rows < 0 || rows > (int64_t(1) << 40) || bad(grad_out) || bad(y) || bad(grad_in) || bad(bias_partial))
    return VSS_E_ARG;
  if (!tanh_grad_cols_ok(cols)) return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const dim3 grid((unsigned)vupd::n_blocks(rows, cols)), block(vupd::kThreads);
  hipStream_t s = (hipStream_t)stream;
  auto g4 = reinterpret_cast<const float4*>(grad_out);
  auto y4 = reinterpret_cast<const float4*>(y);
  auto z4 = reinterpret_cast<float4*>(grad_in);
  auto p4 = reinterpret_cast<float4*>(bias_partial);
  switch (cols) {
    case 64: hipLaunchKernelGGL(vupd::tanh_grad_bias_kernel<16>, grid, block, 0, s, rows, g4, y4, z4, p4); break;
    case 128: hipLaunchKernelGGL(vupd::tanh_grad_bias_kernel<32>, grid, block, 0, s, rows, g4, y4, z4, p4); break;
    case 256: hipLaunchKernelGGL(vupd::tanh_grad_bias_kernel<64>, grid, block, 0, s, rows, g4, y4, z4, p4); break;
    case 512: hipLaunchKernelGGL(vupd::tanh_grad_bias_kernel<128>, grid, block, 0, s, rows, g4, y4, z4, p4); break;
    default: hipLaunchKernelGGL(vupd::tanh_grad_bias_kernel<256>, grid, block, 0, s, rows, g4, y4, z4, p4); break;
  }
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
