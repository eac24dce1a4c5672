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

template <int NA>
__global__ __launch_bounds__(kThreads) void loss_rows_kernel(int64_t rows, int64_t rows_pad, const float* __restrict__ mean,
                                                             const float* __restrict__ logstd, const float* __restrict__ value,
                                                             const float* __restrict__ action, const float* __restrict__ logp_old,
                                                             const float* __restrict__ adv, const float* __restrict__ ret,
                                                             const float* __restrict__ val_old, float clip, float lo, float hi,
                                                             float vf_coef, int clip_vloss, float inv_n,
                                                             float* __restrict__ g_mean, float* __restrict__ g_value,
                                                             float* __restrict__ partial) {
  constexpr int K = kFixed + NA;
  __shared__ float red[kThreads / 64][K];
  // the distribution's per-dimension constants, as torch.distributions.Normal forms them from
  // scale = exp(logstd): var = scale^2, log_scale = log(scale)
  float var[NA], lsc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const float s = expf(logstd[a]);
    var[a] = s * s;
    lsc[a] = logf(s);
  }
  const float log_sqrt_2pi = 0.91893853320467274178f;  // math.log(math.sqrt(2 * math.pi)) as fp32
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < rows_pad; r += stride) {
    if (r >= rows) {  // padding rows: no loss term, no gradient (and no input read)
#pragma unroll
      for (int a = 0; a < NA; ++a) g_mean[r * NA + a] = 0.f;
      g_value[r] = 0.f;
      continue;
    }
    float mu[NA], x[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      mu[a] = mean[r * NA + a];
      x[a] = action[r * NA + a];
    }
    float nlp = 0.f;
    float dz[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      dz[a] = x[a] - mu[a];
      nlp += -(dz[a] * dz[a]) / (2.f * var[a]) - lsc[a] - log_sqrt_2pi;
    }
    const float logratio = nlp - logp_old[r];
    const float ratio = expf(logratio);
    const float A = adv[r];
    acc[2] += -logratio;
    acc[3] += (ratio - 1.f) - logratio;
    acc[4] += fabsf(ratio - 1.f) > clip ? 1.f : 0.f;
    const bool in_r = ratio >= lo && ratio <= hi;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float p1 = -A * ratio, p2 = -A * rc;
    acc[0] += fmaxf(p1, p2);
    const float w1 = p1 > p2 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
    const float w2 = p2 > p1 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
    const float dratio = w1 * -A + (in_r ? w2 * -A : 0.f);
    const float dnlp = dratio * ratio;  // x inv_n for the per-row gradient
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      g_mean[r * NA + a] = dnlp * inv_n * (dz[a] / var[a]);
      acc[kFixed + a] += dnlp * ((dz[a] * dz[a]) / var[a] - 1.f);
    }
    const float v = value[r], R = ret[r];
    float dv;
    if (clip_vloss) {
      const float vo = val_old[r];
      const float d = v - vo;
      const float vc = vo + fminf(fmaxf(d, -clip), clip);
      const float eu = v - R, ec = vc - R;
      const float lu = eu * eu, lc = ec * ec;
      acc[1] += fmaxf(lu, lc);
      const float wu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
      const float wc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
      const bool in_v = d >= -clip && d <= clip;
      dv = 0.5f * (wu * 2.f * eu + (in_v ? wc * 2.f * ec : 0.f));
    } else {
      const float e = v - R;
      acc[1] += e * e;
      dv = e;  // 0.5 x 2 (v - R)
    }
    g_value[r] = vf_coef * dv * inv_n;
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
    partial[(int64_t)blockIdx.x * K + threadIdx.x] = s;
  }
}

// one block: the partial rows summed in block order (deterministic), then the losses, the statistics
// and the log-std gradient.  loss_out[0] = loss; stats_out = [pg_loss, v_loss, entropy_loss,
// old_approx_kl, approx_kl, clipfrac]
template <int NA>
__global__ __launch_bounds__(kThreads) void loss_finish_kernel(int blocks, const float* __restrict__ logstd,
                                                               float ent_coef, float vf_coef, float n, float inv_n,
                                                               const float* __restrict__ partial,
                                                               float* __restrict__ g_logstd, float* __restrict__ loss_out,
                                                               float* __restrict__ stats) {
  constexpr int K = kFixed + NA;
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
  }
}

static int64_t blocks_for(int64_t rows_pad) {
  int64_t b = (rows_pad + kThreads - 1) / kThreads;
  return b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b);
}

template <int NA>
static int launch(void* stream, int64_t rows, int64_t rows_pad, const float* mean, const float* logstd,
                  const float* value, const float* action, const float* logp_old, const float* adv, const float* ret,
                  const float* val_old, float clip, float lo, float hi, float ent_coef, float vf_coef, int clip_vloss,
                  float* g_mean, float* g_value, float* g_logstd, float* loss_out, float* stats, float* partial) {
  const int64_t blocks = blocks_for(rows_pad);
  const float inv_n = 1.0f / (float)rows;
  hipLaunchKernelGGL(loss_rows_kernel<NA>, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, rows,
                     rows_pad, mean, logstd, value, action, logp_old, adv, ret, val_old, clip, lo, hi, vf_coef,
                     clip_vloss, inv_n, g_mean, g_value, partial);
  if (hipGetLastError() != hipSuccess) return VSS_E_LAUNCH;
  hipLaunchKernelGGL(loss_finish_kernel<NA>, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, (int)blocks, logstd,
                     ent_coef, vf_coef, (float)rows, inv_n, partial, g_logstd, loss_out, stats);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
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
  switch (n_act) {
#define VSS_LOSS_CASE(NA)                                                                                         \
  case NA:                                                                                                        \
    return vloss::launch<NA>(stream, rows, rows_pad, mean, logstd, value, action, logprob_old, adv, returns,      \
                             values_old, clip_coef, clip_lo, clip_hi, ent_coef, vf_coef, clip_vloss, grad_mean,  \
                             grad_value, grad_logstd, loss_out, stats_out, partial);
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

}  // extern "C"
