// vss_optim.hip — the PPO update's gradient bookkeeping around the GEMMs (gfx950).
//
// SURVEY §8 A13 (ppo_continuous_action_isaacgym.py:351-354): after loss.backward() the reference clips the
// gradient norm (nn.utils.clip_grad_norm_, ppo…:353) and steps Adam (optim.Adam(eps=1e-5), ppo…:166,354).
// Here every parameter and every gradient of the Agent lives in one flat fp32 buffer
// (vss_amd/flat.py FlatGrads / FlatAdam), so both are two launches over 1.07 M floats
// instead of torch's per-tensor norm chain + multi-tensor Adam (~8 launches, ~130 us per minibatch at the
// reference's 4,095 envs, profiles/r05_ppo_4095_minibatch_window.txt):
//
//   vss_grad_sq_partials:  partial[b] = sum of g^2 over block b's chunk (fixed order: deterministic)
//   vss_adam_step_clipped: every block sums the partials (same fixed order), norm = sqrt, the clip
//                          coefficient min(1, max_norm / (norm + 1e-6)) of clip_grad_norm_, g *= coef
//                          (written back, as clip_grad_norm_ leaves the gradients), then Adam's update
//                          with torch's fused-Adam arithmetic (bias corrections from the step count).
//
// And the split GEMMs' partial sums (weight gradients over row parts, bias-gradient column sums) are
// reduced for a whole MLP backward in ONE launch (vss_sum_parts: a list of jobs, each dst[r][c] = the sum
// over its parts of src[s][r][c], in a fixed order) instead of one torch.sum per tensor.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/vss.h"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_optim.hip targets gfx950 (CDNA4) only"
#endif

namespace vopt {

constexpr int kThreads = 256;
constexpr int kMaxPartials = 1024;  // norm partial blocks (each block of the step kernel re-reads them)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// block sum in a fixed order: lanes, then the 4 waves in order
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float t = red[0];
#pragma unroll
  for (int w = 1; w < kThreads / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

// block b owns elements [b chunk, (b + 1) chunk); within it thread t the strided elements t, t + 256, ...
__global__ __launch_bounds__(kThreads) void sq_partials_kernel(int64_t n, int64_t chunk, const float* __restrict__ g,
                                                                 float* __restrict__ partial) {
  __shared__ float red[kThreads / 64];
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    const float x = g[i];
    s = fmaf(x, x, s);
  }
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(kThreads) void adam_step_kernel(int64_t n, int32_t nparts, const float* __restrict__ partial,
                                                               float max_norm, float lr, float beta1, float beta2, float eps,
                                                               float step, float* __restrict__ g, float* __restrict__ p,
                                                               float* __restrict__ m, float* __restrict__ v,
                                                               float* __restrict__ norm_out) {
  __shared__ float red[kThreads / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kThreads) s += partial[i];
  const float sq = block_sum(s, red);
  const float norm = sqrtf(sq);
  float coef = 1.f;
  const bool clip = max_norm >= 0.f;  // < 0: no clip requested (0 is a clip to zero, as clip_grad_norm_'s)
  if (clip) {  // clip_grad_norm_: clip_coef = max_norm / (total_norm + 1e-6), clamped to 1
    const float c = max_norm / (norm + 1e-6f);
    coef = c < 1.f ? c : 1.f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = norm;
  // torch's fused Adam (opmath fp32): bias corrections from the step count
  const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    float gi = g[i];
    if (clip) {
      gi = gi * coef;
      g[i] = gi;
    }
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * mi / denom;
  }
}

// one launch for many partial-sum reductions: job q owns blocks [first[q], first[q + 1]) of a 1-D grid
// (no idle blocks for the short jobs)
struct PartJob {
  const float* src;
  float* dst;
  int64_t parts, part_stride, rows, cols, src_ld, dst_ld;
  int32_t vec;  // 4: 16-B aligned rows and strides, 4 consecutive columns per lane (float4 loads)
};
constexpr int kMaxPartJobs = 32;
struct PartJobs {
  PartJob j[kMaxPartJobs];
  int32_t first[kMaxPartJobs + 1];
  int32_t count;
};

// a block takes 64 lanes x V consecutive output elements; its 4 waves split the parts (wave w: parts
// w, w + 4, ...), each lane with 8 independent running sums so that 8 loads are in flight, then the 8 sums,
// and the 4 waves' sums through LDS, are added in a fixed order (deterministic).  The bias column sums
// (128-256 parts of 256-512 elements) are then latency-parallel, not one serial chain per column: round 4's
// one-thread-per-column form of this launch was slower than torch's separate sums.
template <int V>
__device__ __forceinline__ void sum_parts_job(const PartJob& J, int64_t blk, float (*red)[64 * 4]) {
  typedef float fv __attribute__((ext_vector_type(V)));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t len = J.rows * J.cols, e = (blk * 64 + lane) * V;
  fv a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = (fv)(0.f);
  if (e < len) {
    const int64_t r = e / J.cols, c = e - r * J.cols;  // V | cols: the lane's V columns share one row
    const float* s = J.src + r * J.src_ld + c;
    int64_t q = wv;
    for (; q + 28 < J.parts; q += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += *reinterpret_cast<const fv*>(s + (q + 4 * u) * J.part_stride);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (q + 4 * u < J.parts) a[u] += *reinterpret_cast<const fv*>(s + (q + 4 * u) * J.part_stride);
  }
  const fv t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
  for (int v = 0; v < V; ++v) red[wv][lane * V + v] = t[v];
  __syncthreads();
  if (wv == 0 && e < len) {
    const int64_t r = e / J.cols, c = e - r * J.cols;
    fv o;
#pragma unroll
    for (int v = 0; v < V; ++v)
      o[v] = (red[0][lane * V + v] + red[1][lane * V + v]) + (red[2][lane * V + v] + red[3][lane * V + v]);
    *reinterpret_cast<fv*>(J.dst + r * J.dst_ld + c) = o;
  }
}

__global__ __launch_bounds__(kThreads) void sum_parts_kernel(PartJobs jobs) {
  __shared__ float red[kThreads / 64][64 * 4];
  const int b = (int)blockIdx.x;
  int q = 0;
  while (q + 1 < jobs.count && jobs.first[q + 1] <= b) ++q;
  const PartJob& J = jobs.j[q];
  if (J.vec == 4) sum_parts_job<4>(J, b - jobs.first[q], red);
  else sum_parts_job<1>(J, b - jobs.first[q], red);
}

static int blocks_for(int64_t n, int64_t per) {
  int64_t b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace vopt

extern "C" {

int64_t vss_grad_sq_partials_count(int64_t n) {
  if (n <= 0) return -1;
  // chunks of at least 4,096 elements, at most kMaxPartials of them
  int64_t b = (n + 4095) / 4096;
  if (b > vopt::kMaxPartials) b = vopt::kMaxPartials;
  return b;
}

int vss_grad_sq_partials(void* stream, int64_t n, const float* grad, float* partial) {
  const int64_t nb = vss_grad_sq_partials_count(n);
  if (nb < 0 || !grad || !partial) return VSS_E_ARG;
  const int64_t chunk = (n + nb - 1) / nb;
  hipLaunchKernelGGL(vopt::sq_partials_kernel, dim3((unsigned)nb), dim3(vopt::kThreads), 0, (hipStream_t)stream, n, chunk,
                     grad, partial);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_adam_step_clipped(void* stream, int64_t n, int32_t nparts, const float* partial, float max_norm, float lr,
                          float beta1, float beta2, float eps, int64_t step, float* grad, float* param, float* exp_avg,
                          float* exp_avg_sq, float* norm_out) {
  if (n <= 0 || nparts < 1 || nparts > vopt::kMaxPartials || !partial || !grad || !param || !exp_avg || !exp_avg_sq ||
      step < 1 || !(eps >= 0.f) || !(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f))
    return VSS_E_ARG;
  int blocks = vopt::blocks_for(n, 4 * vopt::kThreads);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(vopt::adam_step_kernel, dim3((unsigned)blocks), dim3(vopt::kThreads), 0, (hipStream_t)stream, n,
                     nparts, partial, max_norm, lr, beta1, beta2, eps, (float)step, grad, param, exp_avg, exp_avg_sq,
                     norm_out);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_sum_parts(void* stream, int32_t count, const float* const* src, float* const* dst, const int64_t* parts,
                  const int64_t* part_stride, const int64_t* rows, const int64_t* cols, const int64_t* src_ld,
                  const int64_t* dst_ld) {
  if (count < 1 || count > vopt::kMaxPartJobs || !src || !dst || !parts || !part_stride || !rows || !cols || !src_ld ||
      !dst_ld)
    return VSS_E_ARG;
  vopt::PartJobs jobs{};
  int64_t total = 0;
  for (int q = 0; q < count; ++q) {
    if (!src[q] || !dst[q] || parts[q] < 1 || rows[q] < 1 || cols[q] < 1 || src_ld[q] < cols[q] ||
        dst_ld[q] < cols[q] || (parts[q] > 1 && part_stride[q] < rows[q] * src_ld[q] - (src_ld[q] - cols[q])))
      return VSS_E_ARG;
    const bool v4 = cols[q] % 4 == 0 && src_ld[q] % 4 == 0 && dst_ld[q] % 4 == 0 && part_stride[q] % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(src[q]) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst[q]) & 15) == 0;
    jobs.j[q] = vopt::PartJob{src[q], dst[q], parts[q], part_stride[q], rows[q], cols[q], src_ld[q], dst_ld[q], v4 ? 4 : 1};
    const int64_t nb = (rows[q] * cols[q] + 64 * jobs.j[q].vec - 1) / (64 * jobs.j[q].vec);  // 64 lanes x V
    jobs.first[q] = (int32_t)total;
    total += nb;
    if (total > (1 << 24)) return VSS_E_ARG;
  }
  jobs.first[count] = (int32_t)total;
  jobs.count = count;
  hipLaunchKernelGGL(vopt::sum_parts_kernel, dim3((unsigned)total), dim3(vopt::kThreads), 0, (hipStream_t)stream, jobs);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
