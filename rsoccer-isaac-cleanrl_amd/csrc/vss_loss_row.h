// vss_loss_row.h — the per-row terms of the clipped PPO loss (ppo_continuous_action_isaacgym.py:318-349),
// shared by vss_loss.hip (the two-launch loss) and vss_gemm_x6.hip (the loss folded into the output
// layers' forward epilogue) so both evaluate the same fp32 expressions in the same order.
#pragma once

namespace vlossrow {

// the loss sums one block of the x6 GEMM's fused loss epilogue (vss_gemm_x6.hip EPI_LOSS_*) writes,
// 32 floats per block: [0] policy surrogate, [1] value error term, [2] -logratio, [3] (ratio - 1) - logratio,
// [4] clipped count, actor: [5 + a] the log-std gradient's terms, [5 + NA + a] the mean gradients (the
// output bias's gradient); critic: [5] the value gradients (the value bias's gradient)
constexpr int kBlockStats = 32;


constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // math.log(math.sqrt(2 * math.pi)) as fp32

// torch.distributions.Normal's per-dimension constants from scale = exp(logstd): var = scale^2,
// log_scale = log(scale)
template <int NA>
__device__ __forceinline__ void actor_consts(const float* logstd, float (&var)[NA], float (&lsc)[NA]) {
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const float s = expf(logstd[a]);
    var[a] = s * s;
    lsc[a] = logf(s);
  }
}

// one row's policy terms: newlogprob = sum_a Normal(mu, scale).log_prob(x), the ratio to logp_old, the
// clipped surrogate max(-A ratio, -A clamp(ratio)) with torch's conventions at the kinks (maximum splits a
// tie in half, clamp passes [lo, hi]); out: pg, -logratio, (ratio - 1) - logratio, the clip indicator, the
// per-row mean gradient gm[a] (x inv_n) and the log-std gradient term lg[a] (summed, then x inv_n)
template <int NA>
__device__ __forceinline__ void actor_row(const float (&mu)[NA], const float (&x)[NA], float logp_old, float A,
                                          const float (&var)[NA], const float (&lsc)[NA], float clip, float lo,
                                          float hi, float inv_n, float& pg, float& nlr, float& kl, float& cf,
                                          float (&gm)[NA], float (&lg)[NA]) {
  float nlp = 0.f;
  float dz[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    dz[a] = x[a] - mu[a];
    nlp += -(dz[a] * dz[a]) / (2.f * var[a]) - lsc[a] - kLogSqrt2Pi;
  }
  const float logratio = nlp - logp_old;
  const float ratio = expf(logratio);
  nlr = -logratio;
  kl = (ratio - 1.f) - logratio;
  cf = fabsf(ratio - 1.f) > clip ? 1.f : 0.f;
  const bool in_r = ratio >= lo && ratio <= hi;
  const float rc = fminf(fmaxf(ratio, lo), hi);
  const float p1 = -A * ratio, p2 = -A * rc;
  pg = fmaxf(p1, p2);
  const float w1 = p1 > p2 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
  const float w2 = p2 > p1 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
  const float dratio = w1 * -A + (in_r ? w2 * -A : 0.f);
  const float dnlp = dratio * ratio;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    gm[a] = dnlp * inv_n * (dz[a] / var[a]);
    lg[a] = dnlp * ((dz[a] * dz[a]) / var[a] - 1.f);
  }
}

// one row's value terms: 0.5 (v - R)^2, or with clip_vloss the max of that and the clipped value's loss;
// out: the squared-error term vl (summed, then 0.5 / n) and the per-row gradient gv (x vf_coef x inv_n)
__device__ __forceinline__ void critic_row(float v, float R, float vo, int clip_vloss, float clip, float vf_coef,
                                           float inv_n, float& vl, float& gv) {
  float dv;
  if (clip_vloss) {
    const float d = v - vo;
    const float vc = vo + fminf(fmaxf(d, -clip), clip);
    const float eu = v - R, ec = vc - R;
    const float lu = eu * eu, lc = ec * ec;
    vl = fmaxf(lu, lc);
    const float wu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
    const float wc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
    const bool in_v = d >= -clip && d <= clip;
    dv = 0.5f * (wu * 2.f * eu + (in_v ? wc * 2.f * ec : 0.f));
  } else {
    const float e = v - R;
    vl = e * e;
    dv = e;  // 0.5 x 2 (v - R)
  }
  gv = vf_coef * dv * inv_n;
}

}  // namespace vlossrow
