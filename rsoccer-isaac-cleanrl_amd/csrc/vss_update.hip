// vss_update.hip — PPO-update helper on gfx950 (ppo_continuous_action_isaacgym.py:306-353).
//
// The update back-propagates through the Agent's tanh MLPs (ppo…:104-125).  For each hidden
// layer torch issues two memory-bound passes over the (rows x cols) gradient: tanh_backward
// (gz = gy * (1 - y^2): read gy, y, write gz) and the bias gradient (db = sum over rows of gz:
// read gz again).  This kernel does both in one pass: every workgroup owns a chunk of
// kChunkRows rows, writes gz and one row of per-chunk column sums; the caller reduces the
// (chunks x cols) partial sums (a few MB) to db.  Row chunks and the order of the sums are
// fixed, so db is deterministic.  HBM bytes per element: 12 (gy, y read, gz write) instead of 16.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"

namespace vupd {

constexpr int kThreads = 256;
constexpr int64_t kChunkRows = 1024;

__device__ __forceinline__ float4 tanh_grad(float4 g, float4 y) {
  // d tanh(z) / dz = 1 - tanh(z)^2
  return make_float4(g.x * fmaf(-y.x, y.x, 1.0f), g.y * fmaf(-y.y, y.y, 1.0f), g.z * fmaf(-y.z, y.z, 1.0f),
                     g.w * fmaf(-y.w, y.w, 1.0f));
}

__device__ __forceinline__ void add4(float4& a, float4 b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// C4 = cols / 4 float4 columns; RG = kThreads / C4 rows in flight per workgroup step.  Lane t
// owns float4 column t % C4 of rows rg, rg + RG, ... of the chunk (coalesced: a wave reads
// contiguous 16-B words of one or more whole rows).  Up to 4 waves per SIMD: the register budget
// then holds all 2U loads of a lane in flight (at 8 waves the compiler caps it at 64 VGPRs and
// serialises the loads behind the stores).
template <int C4>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 4))) void tanh_grad_bias_kernel(int64_t rows, const float4* __restrict__ gy,
                                                                  const float4* __restrict__ y, float4* __restrict__ gz,
                                                                  float4* __restrict__ partial) {
  constexpr int RG = kThreads / C4;
  static_assert(RG * C4 == kThreads, "cols / 4 must divide the workgroup size");
  __shared__ float4 red[kThreads];
  const int t = threadIdx.x, c4 = t % C4, rg = t / C4;
  const int64_t r0 = (int64_t)blockIdx.x * kChunkRows;
  const int64_t r1 = rows < r0 + kChunkRows ? rows : r0 + kChunkRows;
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int64_t r = r0 + rg;
  constexpr int U = 8;  // rows per lane in flight (16 x 16-B loads per lane before the first use)
  for (; r + (U - 1) * RG < r1; r += U * RG) {
    const int64_t base = r * C4 + c4;
    const float4* pg = gy + base;
    const float4* py = y + base;
    float4* pz = gz + base;
    float4 g[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      g[u] = pg[u * RG * C4];
      v[u] = py[u * RG * C4];
    }
    __builtin_amdgcn_sched_barrier(0);  // all 2U loads issued before the first store
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float4 z = tanh_grad(g[u], v[u]);
      pz[u * RG * C4] = z;
      add4(acc, z);
    }
  }
  for (; r < r1; r += RG) {
    const int64_t i = r * C4 + c4;
    const float4 z = tanh_grad(gy[i], y[i]);
    gz[i] = z;
    add4(acc, z);
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

int64_t vss_tanh_grad_chunks(int64_t rows) {
  return rows < 0 ? -1 : (rows + vupd::kChunkRows - 1) / vupd::kChunkRows;
}

int vss_tanh_grad_bias(void* stream, int64_t rows, int32_t cols, const float* grad_out, const float* y,
                       float* grad_in, float* bias_partial) {
  auto bad = [](const void* p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) != 0; };
  if (rows < 0 || rows > (int64_t(1) << 40) || bad(grad_out) || bad(y) || bad(grad_in) || bad(bias_partial))
    return VSS_E_ARG;
  if (!(cols == 64 || cols == 128 || cols == 256 || cols == 512 || cols == 1024)) return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const dim3 grid((unsigned)vss_tanh_grad_chunks(rows)), block(vupd::kThreads);
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
