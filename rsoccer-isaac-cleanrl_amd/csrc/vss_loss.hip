// vss_loss.hip — the clipped PPO loss of one update minibatch and its gradients, in two launches (gfx950).
//
// SURVEY §8 A13, ppo_continuous_action_isaacgym.py:314-349 (cleanrl's clipped surrogate): from the
// actor's output (means), the shared log-std, the critic's output and the rollout's stored
// action / log-prob / advantage / return / value of every minibatch row,
//   newlogprob = sum_a Normal(mean, exp(logstd)).log_prob(action)       (torch.distributions.Normal)
//   logratio = newlogprob - logprob_old, ratio = exp(logratio)
//   old_approx_kl = mean(-logratio), approx_kl = mean((ratio - 1) - logratio),
//   clipfrac = mean(|ratio - 1| > clip)
//   pg_loss = mean(max(-adv ratio, -adv clamp(ratio, 1 - clip, 1 + clip)))
//   v_loss = 0.5 mean((v - R)^2), or with clip_vloss 0.5 mean(max((v - R)^2, (val + clamp(v - val,
//            -clip, clip) - R)^2))
//   entropy_loss = mean(sum_a (0.5 + 0.5 log 2 pi + log scale_a))
//   loss = pg_loss - ent_coef entropy_loss + vf_coef v_loss
// and the loss's gradients with respect to the means, the values and the log-std, with torch's
// autograd conventions for the non-smooth points (torch.maximum splits the gradient in half on a tie,
// torch.clamp passes it on the closed interval [lo, hi]).  Torch runs this as ~100 small kernels per
// minibatch (forward and backward); here one grid-stride pass writes the per-row gradients and one
// block-partial row of sums per block, and a one-block pass reduces the partials in a fixed order
// (deterministic) into the losses, the statistics and the log-std gradient.  Rows r in [rows, rows_pad)
// (the update's padding rows, copies that the losses must not see) get zero gradients.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"
#include "vss_loss_row.h"
#include <hipcub/hipcub.hpp>

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_loss.hip targets gfx950 (CDNA4) only"
#endif

namespace vloss {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;
// partial sums per block: pg, v, -logratio, (ratio - 1) - logratio, clipped count, then per action dim
// sum_i dratio_i ratio_i ((x - mu)^2 / var - 1)
constexpr int kFixed = 5;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// the direct form (vss_ppo_loss_direct) reads the networks' outputs as the output layers' epilogue parts
// and the raw advantages with their normalisation sums, and also sums the output biases' gradients
struct RowsArgs {
  int64_t rows, rows_pad;
  const float* mean;   // (rows_pad, NA); DIRECT: mparts x (rows_pad, NA) epilogue parts of the actor's output
  const float* value;  // (rows_pad,);    DIRECT: vparts x (rows_pad,) parts of the critic's output
  int mparts, vparts;
  const float* b_mean;  // DIRECT: the output layers' biases (NA,) and (1,)
  const float* b_value;
  const double* adv_part;  // DIRECT, or NULL: nparts x (sum, sum of squares) of the raw advantages
  int adv_nparts;
  double adv_count;
  const float* logstd;
  const float* action;
  const float* logp_old;
  const float* adv;
  const float* ret;
  const float* val_old;
  float clip, lo, hi, vf_coef;
  int clip_vloss;
  float inv_n;
  float* g_mean;
  float* g_value;
  float* partial;
};

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// (sum, sum of squares) parts of the advantages -> (mean, std) as fp32, the fp64 formula of
// normalize_advantages' all-reduced branch (vss_amd/minibatch.py): mean = s / n,
// std = sqrt(max((q - n mean mean) / (n - 1), 0)).  Every block the same fixed order: wave 0's lanes
// take parts lane, lane + 64, ..., then the wave sum; the result is shared through LDS.
__device__ __forceinline__ void adv_moments(const double* part, int nparts, double n, float& mean, float& std) {
  __shared__ float mom[2];
  if (threadIdx.x < 64) {
    double s = 0.0, q = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 64) {
      s += part[2 * i];
      q += part[2 * i + 1];
    }
    s = wave_sum_f64(s);
    q = wave_sum_f64(q);
    if (threadIdx.x == 0) {
      const double m = s / n;
      double var = (q - n * m * m) / (n - 1.0);
      var = var > 0.0 ? var : 0.0;
      mom[0] = (float)m;
      mom[1] = (float)sqrt(var);
    }
  }
  __syncthreads();
  mean = mom[0];
  std = mom[1];
}

template <int NA, bool DIRECT>
__global__ __launch_bounds__(kThreads) void loss_rows_kernel(const RowsArgs p) {
  // DIRECT also sums the per-row gradients of the actor's means (NA) and of the value (1): the output
  // layers' bias gradients
  constexpr int K = kFixed + NA + (DIRECT ? NA + 1 : 0);
  __shared__ float red[kThreads / 64][K];
  const int64_t rows = p.rows, rows_pad = p.rows_pad;
  float var[NA], lsc[NA], bm[NA];
  vlossrow::actor_consts<NA>(p.logstd, var, lsc);
#pragma unroll
  for (int a = 0; a < NA; ++a) bm[a] = DIRECT ? p.b_mean[a] : 0.f;
  const float bv = DIRECT ? p.b_value[0] : 0.f;
  float adv_mean = 0.f, adv_std = 0.f;
  const bool norm = DIRECT && p.adv_part != nullptr;
  if (norm) adv_moments(p.adv_part, p.adv_nparts, p.adv_count, adv_mean, adv_std);
  const float inv_n = p.inv_n, clip = p.clip, lo = p.lo, hi = p.hi;
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < rows_pad; r += stride) {
    if (r >= rows) {  // padding rows: no loss term, no gradient (and no input read)
#pragma unroll
      for (int a = 0; a < NA; ++a) p.g_mean[r * NA + a] = 0.f;
      p.g_value[r] = 0.f;
      continue;
    }
    float mu[NA], x[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      if constexpr (DIRECT) {  // the output layer's parts, in order, then its bias
        float m = p.mean[r * NA + a];
        for (int q = 1; q < p.mparts; ++q) m += p.mean[((int64_t)q * rows_pad + r) * NA + a];
        mu[a] = m + bm[a];
      } else {
        mu[a] = p.mean[r * NA + a];
      }
      x[a] = p.action[r * NA + a];
    }
    float A = p.adv[r];
    if (norm) A = (A - adv_mean) / (adv_std + 1e-8f);
    float pg, nlr, kl, cf, gm[NA], lg[NA];
    vlossrow::actor_row<NA>(mu, x, p.logp_old[r], A, var, lsc, clip, lo, hi, inv_n, pg, nlr, kl, cf, gm, lg);
    acc[0] += pg;
    acc[2] += nlr;
    acc[3] += kl;
    acc[4] += cf;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      p.g_mean[r * NA + a] = gm[a];
      acc[kFixed + a] += lg[a];
      if constexpr (DIRECT) acc[kFixed + NA + a] += gm[a];
    }
    float v;
    if constexpr (DIRECT) {
      v = p.value[r];
      for (int q = 1; q < p.vparts; ++q) v += p.value[(int64_t)q * rows_pad + r];
      v += bv;
    } else {
      v = p.value[r];
    }
    float vl, gv;
    vlossrow::critic_row(v, p.ret[r], p.clip_vloss ? p.val_old[r] : 0.f, p.clip_vloss, clip, p.vf_coef, inv_n, vl, gv);
    acc[1] += vl;
    p.g_value[r] = gv;
    if constexpr (DIRECT) acc[kFixed + 2 * NA] += gv;
  }
  // block reduction: wave sums, then the 4 waves' rows in order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s = wave_sum(acc[k]);
    if (lane == 0) red[wv][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    float s = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kThreads / 64; ++w) s += red[w][threadIdx.x];
    p.partial[(int64_t)blockIdx.x * K + threadIdx.x] = s;
  }
}

// one block: the partial rows summed in block order (deterministic), then the losses, the statistics
// and the log-std gradient.  loss_out[0] = loss; stats_out = [pg_loss, v_loss, entropy_loss,
// old_approx_kl, approx_kl, clipfrac]
template <int NA, bool DIRECT>
__global__ __launch_bounds__(kThreads) void loss_finish_kernel(int blocks, const float* __restrict__ logstd,
                                                               float ent_coef, float vf_coef, float n, float inv_n,
                                                               const float* __restrict__ partial,
                                                               float* __restrict__ g_logstd, float* __restrict__ loss_out,
                                                               float* __restrict__ stats, float* __restrict__ db_mean,
                                                               float* __restrict__ db_value) {
  constexpr int K = kFixed + NA + (DIRECT ? NA + 1 : 0);
  __shared__ float tot[K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // wave wv sums quantities k = wv, wv + 4, ...: lanes stride over the blocks, then a wave sum
  for (int k = wv; k < K; k += kThreads / 64) {
    float s = 0.f;
    for (int b = lane; b < blocks; b += 64) s += partial[(int64_t)b * K + k];
    s = wave_sum(s);
    if (lane == 0) tot[k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ent = 0.f;
#pragma unroll
    for (int a = 0; a < NA; ++a) ent += 1.41893853320467274178f + logf(expf(logstd[a]));  // 0.5 + 0.5 log(2 pi), as one fp32 constant
    // means as torch forms them (the sum divided by the count)
    const float pg = tot[0] / n, vl = 0.5f * (tot[1] / n);
    loss_out[0] = pg - ent_coef * ent + vl * vf_coef;
    stats[0] = pg;
    stats[1] = vl;
    stats[2] = ent;
    stats[3] = tot[2] / n;
    stats[4] = tot[3] / n;
    stats[5] = tot[4] / n;
#pragma unroll
    for (int a = 0; a < NA; ++a) g_logstd[a] = tot[kFixed + a] * inv_n - ent_coef;
    if constexpr (DIRECT) {
#pragma unroll
      for (int a = 0; a < NA; ++a) db_mean[a] = tot[kFixed + NA + a];
      db_value[0] = tot[kFixed + 2 * NA];
    }
  }
}

// the fused loss epilogue's per-block sums (vss_gemm_x6.hip EPI_LOSS_A / EPI_LOSS_C, vlossrow::kBlockStats
// layout) -> the loss, its statistics, the log-std gradient and the output biases' gradients, as
// loss_finish_kernel<NA, true> forms them
constexpr int kFinishThreads = 1024;
template <int NA>
__global__ __launch_bounds__(kFinishThreads) void fused_finish_kernel(int actor_blocks, const float* __restrict__ actor,
                                                                int critic_blocks, const float* __restrict__ critic,
                                                                const float* __restrict__ logstd, float ent_coef,
                                                                float vf_coef, float n, float inv_n,
                                                                float* __restrict__ g_logstd, float* __restrict__ loss_out,
                                                                float* __restrict__ stats, float* __restrict__ db_mean,
                                                                float* __restrict__ db_value) {
  // thread t: quantity k = t % 64 (actor's 32, then the critic's), block chunk c = t / 64 of kFinishThreads / 64:
  // its blocks c, c + 16, ... summed with all loads in flight at once, then the 16 chunk sums in order
  constexpr int S = vlossrow::kBlockStats, CH = kFinishThreads / 64;
  __shared__ float part[CH][2 * S];
  __shared__ float tot[2 * S];
  {
    const int k = threadIdx.x & 63, ch = threadIdx.x >> 6;
    const bool c = k >= S;
    const float* p = c ? critic : actor;
    const int blocks = c ? critic_blocks : actor_blocks, kk = c ? k - S : k;
    float s = 0.f;
#pragma unroll 8
    for (int b = ch; b < blocks; b += CH) s += p[(int64_t)b * S + kk];
    part[ch][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < 2 * S) {
    float s = part[0][threadIdx.x];
#pragma unroll
    for (int ch = 1; ch < CH; ++ch) s += part[ch][threadIdx.x];
    tot[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float* ta = tot;
    const float* tc = tot + S;
    float ent = 0.f;
#pragma unroll
    for (int a = 0; a < NA; ++a) ent += 1.41893853320467274178f + logf(expf(logstd[a]));
    const float pg = ta[0] / n, vl = 0.5f * (tc[1] / n);
    loss_out[0] = pg - ent_coef * ent + vl * vf_coef;
    stats[0] = pg;
    stats[1] = vl;
    stats[2] = ent;
    stats[3] = ta[2] / n;
    stats[4] = ta[3] / n;
    stats[5] = ta[4] / n;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      g_logstd[a] = ta[kFixed + a] * inv_n - ent_coef;
      db_mean[a] = ta[kFixed + NA + a];
    }
    db_value[0] = tc[kFixed];
  }
}

static int64_t blocks_for(int64_t rows_pad) {
  int64_t b = (rows_pad + kThreads - 1) / kThreads;
  return b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b);
}

template <int NA, bool DIRECT>
static int launch(void* stream, const RowsArgs& a, float ent_coef, float* g_logstd, float* loss_out, float* stats,
                  float* db_mean, float* db_value) {
  const int64_t blocks = blocks_for(a.rows_pad);
  hipLaunchKernelGGL((loss_rows_kernel<NA, DIRECT>), dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  if (hipGetLastError() != hipSuccess) return VSS_E_LAUNCH;
  hipLaunchKernelGGL((loss_finish_kernel<NA, DIRECT>), dim3(1), dim3(kThreads), 0, (hipStream_t)stream, (int)blocks,
                     a.logstd, ent_coef, a.vf_coef, (float)a.rows, a.inv_n, a.partial, g_logstd, loss_out, stats,
                     db_mean, db_value);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

template <bool DIRECT>
static int dispatch(void* stream, int32_t n_act, const RowsArgs& a, float ent_coef, float* g_logstd, float* loss_out,
                    float* stats, float* db_mean, float* db_value) {
  switch (n_act) {
#define VSS_LOSS_CASE(NA) \
  case NA:                \
    return launch<NA, DIRECT>(stream, a, ent_coef, g_logstd, loss_out, stats, db_mean, db_value);
    VSS_LOSS_CASE(1)
    VSS_LOSS_CASE(2)
    VSS_LOSS_CASE(3)
    VSS_LOSS_CASE(4)
    VSS_LOSS_CASE(6)
    VSS_LOSS_CASE(8)
#undef VSS_LOSS_CASE
    default:
      return VSS_E_ARG;
  }
}

// ---- the minibatch's rows (ppo…:310-317: b_obs[mb_inds], b_actions[mb_inds], b_logprobs[mb_inds],
// b_advantages[mb_inds], b_returns[mb_inds], b_values[mb_inds]) in ONE launch, with the advantages'
// (sum, sum of squares) parts for their normalisation (ppo…:325-326), instead of torch's six gathers,
// a cat and the mean / std chain.  Blocks [0, table_blocks) copy the observation and action rows (rows
// r >= mb, the update's padding, repeat the minibatch's rows r - mb, r - mb - mb, ...); blocks after them
// copy the per-row scalars and sum the advantages in fp64, one part per block, in a fixed order.
constexpr int kGatherTableBlocks = 2048;
constexpr int kGatherScalarBlocks = 256;

struct GatherArgs {
  int64_t mb, rows_pad, batch;
  const int64_t* inds;
  int64_t obs_w, act_w;  // floats per observation / action row
  const float* b_obs;
  const float* b_act;
  const float* b_logp;
  const float* b_adv;
  const float* b_ret;
  const float* b_val;
  float* obs;
  float* act;
  float* logp;
  float* adv;
  float* ret;
  float* val;
  double* adv_part;  // (scalar blocks, 2)
  int table_blocks;
};

// source row of minibatch row r (the padding rows repeat the minibatch); -1 for an index outside the batch
__device__ __forceinline__ int64_t src_row(const GatherArgs& g, int64_t r) {
  const int64_t i = g.inds[r < g.mb ? r : (r - g.mb) % g.mb];
  return (i >= 0 && i < g.batch) ? i : -1;
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void gather_kernel(const GatherArgs g) {
  if ((int)blockIdx.x < g.table_blocks) {
    const int64_t stride = (int64_t)g.table_blocks * kThreads;
    const int64_t t0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const float qnan = __builtin_nanf("");
    if constexpr (VEC) {  // observation rows as 16-B chunks
      const int64_t cw = g.obs_w / 4;
      for (int64_t u = t0; u < g.rows_pad * cw; u += stride) {
        const int64_t r = u / cw, c = u - r * cw;
        const int64_t i = src_row(g, r);
        const float4 v = i >= 0 ? reinterpret_cast<const float4*>(g.b_obs + i * g.obs_w)[c]
                                : make_float4(qnan, qnan, qnan, qnan);
        reinterpret_cast<float4*>(g.obs + r * g.obs_w)[c] = v;
      }
    } else {
      for (int64_t u = t0; u < g.rows_pad * g.obs_w; u += stride) {
        const int64_t r = u / g.obs_w, c = u - r * g.obs_w;
        const int64_t i = src_row(g, r);
        g.obs[u] = i >= 0 ? g.b_obs[i * g.obs_w + c] : qnan;
      }
    }
    for (int64_t u = t0; u < g.rows_pad * g.act_w; u += stride) {
      const int64_t r = u / g.act_w, c = u - r * g.act_w;
      const int64_t i = src_row(g, r);
      g.act[u] = i >= 0 ? g.b_act[i * g.act_w + c] : qnan;
    }
    return;
  }
  __shared__ double red[2][kThreads / 64];
  const int b = (int)blockIdx.x - g.table_blocks, nb = (int)gridDim.x - g.table_blocks;
  double s = 0.0, q = 0.0;
  for (int64_t r = (int64_t)b * kThreads + threadIdx.x; r < g.mb; r += (int64_t)nb * kThreads) {
    const int64_t i = src_row(g, r);
    if (i < 0) {
      const float qnan = __builtin_nanf("");
      g.logp[r] = g.adv[r] = g.ret[r] = g.val[r] = qnan;
      s += (double)qnan;
      continue;
    }
    const float a = g.b_adv[i];
    g.logp[r] = g.b_logp[i];
    g.adv[r] = a;
    g.ret[r] = g.b_ret[i];
    g.val[r] = g.b_val[i];
    s += (double)a;
    q += (double)a * (double)a;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  s = wave_sum_f64(s);
  q = wave_sum_f64(q);
  if (lane == 0) {
    red[0][wv] = s;
    red[1][wv] = q;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double t = red[threadIdx.x][0];
#pragma unroll
    for (int w = 1; w < kThreads / 64; ++w) t += red[threadIdx.x][w];
    g.adv_part[2 * b + threadIdx.x] = t;
  }
}

// the parts summed in order into one (sum, sum of squares) pair -- the order adv_moments uses -- for the
// data-parallel all-reduce of the global statistics
__global__ void adv_part_sum_kernel(int nparts, const double* __restrict__ part, double* __restrict__ out) {
  if (threadIdx.x == 0) {
    double s = 0.0, q = 0.0;
    for (int i = 0; i < nparts; ++i) {
      s += part[2 * i];
      q += part[2 * i + 1];
    }
    out[0] = s;
    out[1] = q;
  }
}

static int64_t gather_scalar_blocks(int64_t mb) {
  int64_t b = (mb + kThreads - 1) / kThreads;
  return b < 1 ? 1 : (b > kGatherScalarBlocks ? kGatherScalarBlocks : b);
}


// ---- the epoch's minibatch permutation (ppo…:309, torch.randperm(batch)): a uniformly random
// permutation from one 64-bit seed drawn from the update's generator.  Each index i gets the key
// (b random bits << (64 - b)) | i (b = 32 in the product), with the random bits from splitmix64 of (seed, i); a
// radix sort on the high bits (4 passes for b = 32) orders the indices by their random bits.  Indices whose
// random bits tie (~n^2 / 2^33 pairs at b = 32) would keep index order after the stable sort; a pass over
// the sorted keys shuffles every such run (Fisher-Yates from a second splitmix64 stream), so the order within
// a run is uniform and independent of the keys, and the permutation is uniform -- as torch.randperm, which
// sorts 64-bit keys (8 passes) and then shuffles its duplicate-key runs the same way.  The low 32 bits of the
// sorted keys are the permutation, written in place as int64.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void perm_keys_kernel(int64_t n, int key_bits, const int64_t* __restrict__ seed,
                                                             uint64_t* __restrict__ keys) {
  const uint64_t s = (uint64_t)seed[0];
  const uint64_t mask = ~0ull << (64 - key_bits);  // the top key_bits of the random word, in bits 32 + ..
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const uint64_t r = splitmix64(s + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
    keys[i] = (r & mask) | (uint64_t)i;
  }
}

// the sorted keys' tied runs (equal high halves) shuffled in place: the thread at a run's first position
// (its left neighbour differs, its right one is equal) walks the run and Fisher-Yates-shuffles its low halves.
// The high halves never change, so the neighbour tests read the same values whatever the other runs' threads
// have written so far; runs are disjoint, so every entry has one writer.
__global__ __launch_bounds__(kThreads) void perm_ties_kernel(int64_t n, const int64_t* __restrict__ seed,
                                                             uint64_t* __restrict__ keys) {
  const uint64_t s = (uint64_t)seed[0] ^ 0xD1B54A32D192ED03ull;  // a stream apart from the keys'
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i + 1 < n; i += stride) {
    const uint64_t hi = keys[i] >> 32;
    if ((keys[i + 1] >> 32) != hi || (i > 0 && (keys[i - 1] >> 32) == hi)) continue;
    int64_t end = i + 2;
    while (end < n && (keys[end] >> 32) == hi) ++end;
    for (int64_t t = end - 1; t > i; --t) {  // position t takes a uniform pick among [i, t]
      const uint64_t r = splitmix64(s + (uint64_t)(t + 1) * 0x9E3779B97F4A7C15ull);
      const int64_t j = i + (int64_t)(r % (uint64_t)(t - i + 1));
      const uint64_t a = keys[t], b = keys[j];
      keys[t] = b;
      keys[j] = a;
    }
  }
}

__global__ __launch_bounds__(kThreads) void perm_index_kernel(int64_t n, uint64_t* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) keys[i] &= 0xFFFFFFFFull;
}

static size_t perm_sort_bytes(int64_t n) {
  size_t bytes = 0;
  if (hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n, 32, 64,
                                        (hipStream_t)0) != hipSuccess)
    return 0;
  return bytes;
}

static int64_t perm_grid(int64_t n) {
  const int64_t g = (n + kThreads - 1) / kThreads;
  return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}
}  // namespace vloss

extern "C" {

int64_t vss_ppo_loss_scratch_floats(int64_t rows_pad, int32_t n_act) {
  if (rows_pad <= 0 || n_act < 1 || n_act > 8) return -1;
  return vloss::blocks_for(rows_pad) * (vloss::kFixed + n_act);
}

int vss_ppo_loss(void* stream, int64_t rows, int64_t rows_pad, int32_t n_act, const float* mean, const float* logstd,
                 const float* value, const float* action, const float* logprob_old, const float* adv,
                 const float* returns, const float* values_old, float clip_coef, float clip_lo, float clip_hi,
                 float ent_coef, float vf_coef, int32_t clip_vloss, float* grad_mean, float* grad_value,
                 float* grad_logstd, float* loss_out, float* stats_out, float* partial) {
  if (rows <= 0 || rows_pad < rows || !mean || !logstd || !value || !action || !logprob_old || !adv || !returns ||
      !values_old || !grad_mean || !grad_value || !grad_logstd || !loss_out || !stats_out || !partial)
    return VSS_E_ARG;
  const vloss::RowsArgs a{rows, rows_pad, mean, value, 1, 1, nullptr, nullptr, nullptr, 0, 0.0, logstd, action,
                          logprob_old, adv, returns, values_old, clip_coef, clip_lo, clip_hi, vf_coef, clip_vloss,
                          1.0f / (float)rows, grad_mean, grad_value, partial};
  return vloss::dispatch<false>(stream, n_act, a, ent_coef, grad_logstd, loss_out, stats_out, nullptr, nullptr);
}

int64_t vss_ppo_loss_direct_scratch_floats(int64_t rows_pad, int32_t n_act) {
  if (rows_pad <= 0 || n_act < 1 || n_act > 8) return -1;
  return vloss::blocks_for(rows_pad) * (vloss::kFixed + 2 * n_act + 1);
}

int vss_ppo_loss_direct(void* stream, int64_t rows, int64_t rows_pad, int32_t n_act, const float* mean_parts,
                        int32_t mean_nparts, const float* mean_bias, const float* value_parts, int32_t value_nparts,
                        const float* value_bias, const float* logstd, const float* action, const float* logprob_old,
                        const float* adv, const double* adv_part, int32_t adv_nparts, double adv_count,
                        const float* returns, const float* values_old, float clip_coef, float clip_lo, float clip_hi,
                        float ent_coef, float vf_coef, int32_t clip_vloss, float* grad_mean, float* grad_value,
                        float* grad_logstd, float* grad_mean_bias, float* grad_value_bias, float* loss_out,
                        float* stats_out, float* partial) {
  if (rows <= 0 || rows_pad < rows || mean_nparts < 1 || value_nparts < 1 || !mean_parts || !mean_bias ||
      !value_parts || !value_bias || !logstd || !action || !logprob_old || !adv || !returns || !values_old ||
      !grad_mean || !grad_value || !grad_logstd || !grad_mean_bias || !grad_value_bias || !loss_out || !stats_out ||
      !partial || (adv_part && (adv_nparts < 1 || !(adv_count > 1.0))))
    return VSS_E_ARG;
  const vloss::RowsArgs a{rows, rows_pad, mean_parts, value_parts, mean_nparts, value_nparts, mean_bias, value_bias,
                          adv_part, adv_nparts, adv_count, logstd, action, logprob_old, adv, returns, values_old,
                          clip_coef, clip_lo, clip_hi, vf_coef, clip_vloss, 1.0f / (float)rows, grad_mean, grad_value,
                          partial};
  return vloss::dispatch<true>(stream, n_act, a, ent_coef, grad_logstd, loss_out, stats_out, grad_mean_bias,
                               grad_value_bias);
}

int vss_ppo_loss_fused_finish(void* stream, int64_t rows, int32_t n_act, int64_t actor_blocks, const float* actor_stats,
                              int64_t critic_blocks, const float* critic_stats, const float* logstd, float ent_coef,
                              float vf_coef, float* grad_logstd, float* grad_mean_bias, float* grad_value_bias,
                              float* loss_out, float* stats_out) {
  if (rows <= 0 || actor_blocks < 1 || critic_blocks < 1 || !actor_stats || !critic_stats || !logstd || !grad_logstd ||
      !grad_mean_bias || !grad_value_bias || !loss_out || !stats_out)
    return VSS_E_ARG;
  const dim3 grid(1), block(vloss::kFinishThreads);
  const float n = (float)rows, inv_n = 1.0f / (float)rows;
  if (n_act == 1)
    hipLaunchKernelGGL((vloss::fused_finish_kernel<1>), grid, block, 0, (hipStream_t)stream, (int)actor_blocks,
                       actor_stats, (int)critic_blocks, critic_stats, logstd, ent_coef, vf_coef, n, inv_n, grad_logstd,
                       loss_out, stats_out, grad_mean_bias, grad_value_bias);
  else if (n_act == 2)
    hipLaunchKernelGGL((vloss::fused_finish_kernel<2>), grid, block, 0, (hipStream_t)stream, (int)actor_blocks,
                       actor_stats, (int)critic_blocks, critic_stats, logstd, ent_coef, vf_coef, n, inv_n, grad_logstd,
                       loss_out, stats_out, grad_mean_bias, grad_value_bias);
  else
    return VSS_E_ARG;
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int64_t vss_randperm_scratch_bytes(int64_t n) {
  if (n <= 0 || n > 0xFFFFFFFFll || n > 0x7FFFFFFFll) return -1;
  const size_t sort = vloss::perm_sort_bytes(n);
  if (sort == 0) return -1;
  return ((n * 8 + 255) / 256) * 256 + (int64_t)sort;
}

int vss_randperm_bits(void* stream, int64_t n, int32_t key_bits, const int64_t* seed, int64_t* out, void* scratch,
                      int64_t scratch_bytes) {
  const int64_t need = vss_randperm_scratch_bytes(n);
  if (need < 0 || key_bits < 1 || key_bits > 32 || !seed || !out || !scratch || scratch_bytes < need ||
      (reinterpret_cast<uintptr_t>(scratch) & 255) || (reinterpret_cast<uintptr_t>(out) & 7))
    return VSS_E_ARG;
  uint64_t* keys = static_cast<uint64_t*>(scratch);
  char* temp = static_cast<char*>(scratch) + ((n * 8 + 255) / 256) * 256;
  size_t temp_bytes = (size_t)(scratch_bytes - ((n * 8 + 255) / 256) * 256);
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)vloss::perm_grid(n)), block(vloss::kThreads);
  hipLaunchKernelGGL(vloss::perm_keys_kernel, grid, block, 0, st, n, (int)key_bits, seed, keys);
  if (hipGetLastError() != hipSuccess) return VSS_E_LAUNCH;
  if (hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, reinterpret_cast<uint64_t*>(out), (int)n,
                                        64 - key_bits, 64, st) != hipSuccess)
    return VSS_E_LAUNCH;
  hipLaunchKernelGGL(vloss::perm_ties_kernel, grid, block, 0, st, n, seed, reinterpret_cast<uint64_t*>(out));
  if (hipGetLastError() != hipSuccess) return VSS_E_LAUNCH;
  hipLaunchKernelGGL(vloss::perm_index_kernel, grid, block, 0, st, n, reinterpret_cast<uint64_t*>(out));
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_randperm(void* stream, int64_t n, const int64_t* seed, int64_t* out, void* scratch, int64_t scratch_bytes) {
  return vss_randperm_bits(stream, n, 32, seed, out, scratch, scratch_bytes);
}

int64_t vss_minibatch_gather_parts(int64_t mb) { return mb <= 0 ? -1 : vloss::gather_scalar_blocks(mb); }

int vss_minibatch_gather(void* stream, int64_t mb, int64_t rows_pad, int64_t batch, const int64_t* inds, int64_t obs_w,
                         int64_t act_w, const float* b_obs, const float* b_act, const float* b_logp, const float* b_adv,
                         const float* b_ret, const float* b_val, float* obs, float* act, float* logp, float* adv,
                         float* ret, float* val, double* adv_part) {
  if (mb <= 0 || rows_pad < mb || batch <= 0 || obs_w <= 0 || act_w <= 0 || !inds || !b_obs || !b_act || !b_logp ||
      !b_adv || !b_ret || !b_val || !obs || !act || !logp || !adv || !ret || !val || !adv_part)
    return VSS_E_ARG;
  const int64_t sb = vloss::gather_scalar_blocks(mb);
  const int64_t units = rows_pad * obs_w;
  int64_t tb = (units / 4 + vloss::kThreads - 1) / vloss::kThreads;
  tb = tb < 1 ? 1 : (tb > vloss::kGatherTableBlocks ? vloss::kGatherTableBlocks : tb);
  const vloss::GatherArgs g{mb, rows_pad, batch, inds, obs_w, act_w, b_obs, b_act, b_logp, b_adv, b_ret, b_val, obs, act,
                            logp, adv, ret, val, adv_part, (int)tb};
  const bool vec = obs_w % 4 == 0 && ((reinterpret_cast<uintptr_t>(b_obs) | reinterpret_cast<uintptr_t>(obs)) & 15) == 0;
  const dim3 grid((unsigned)(tb + sb)), block(vloss::kThreads);
  if (vec)
    hipLaunchKernelGGL((vloss::gather_kernel<true>), grid, block, 0, (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL((vloss::gather_kernel<false>), grid, block, 0, (hipStream_t)stream, g);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_adv_part_sum(void* stream, int32_t nparts, const double* part, double* out) {
  if (nparts < 1 || !part || !out) return VSS_E_ARG;
  hipLaunchKernelGGL(vloss::adv_part_sum_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (int)nparts, part, out);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
