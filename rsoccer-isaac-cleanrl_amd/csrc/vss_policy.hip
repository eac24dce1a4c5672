// vss_policy.hip — fused actor/critic MLP forward for PPO rollouts on gfx950.
//
// The reference's Agent (ppo_continuous_action_isaacgym.py:127-164): two MLPs
// 52 -> 256 -> 512 -> 512 -> 256 -> {A | 1}, tanh between layers, a state-independent log-std.
// Per rollout step the reference runs actor + critic on next_obs (ppo…:262) and the critic on
// the terminal observation (ppo…:272): at 65,536 rows that is a GEMM chain (M = 65,536), so it
// runs on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 FMA chains, 157 TF peak).
//
// Layout: one wave = 16 rows (samples).  Every layer is computed transposed,
//   H_out^T (N x 16) = W (N x K) . H_in^T (K x 16),
// so an MFMA accumulator holds 4 output features of one sample per lane (lane l: sample l&15,
// features 16*tile + 4*(l>>4) + r) — exactly the B-operand a following 16x16x4 MFMA needs when
// its k-step (t, r) takes input feature 16t + 4*(l>>4) + r.  Activations therefore stay in
// registers from the first layer to the last (no LDS, no HBM round trips).  The weights are
// repacked once per update (vss_mlp_pack) into that k order and lane order, so each MFMA's A
// operand is one coalesced float4 load (4 output tiles) from L2.  Bias + tanh, the tiny output
// layer (VALU dot products + cross-lane reduction), Gaussian sampling (Philox), log-prob and
// entropy are fused into the epilogue.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"

namespace vpol {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIn = 52, kH1 = 256, kH2 = 512, kH3 = 512, kH4 = 256;
constexpr int kWaves = 4;          // waves per workgroup (independent; 64 rows per workgroup)
constexpr int kRowsPerWave = 16;

// packed-buffer offsets (floats) of one network with n_out outputs
__host__ __device__ constexpr int64_t off_w1() { return 0; }
__host__ __device__ constexpr int64_t off_w2() { return off_w1() + (int64_t)kIn * kH1; }
__host__ __device__ constexpr int64_t off_w3() { return off_w2() + (int64_t)kH1 * kH2; }
__host__ __device__ constexpr int64_t off_w4() { return off_w3() + (int64_t)kH2 * kH3; }
__host__ __device__ constexpr int64_t off_w5() { return off_w4() + (int64_t)kH3 * kH4; }
__host__ __device__ constexpr int64_t off_b(int n_out) { return off_w5() + (int64_t)n_out * kH4; }
__host__ __device__ constexpr int64_t packed_size(int n_out) {
  return off_b(n_out) + kH1 + kH2 + kH3 + kH4 + n_out;
}

// ---- packing ---------------------------------------------------------------------------------------
// MFMA layer (K inputs, N outputs, K4 = K/4 k-steps, NT = N/16 output tiles), packed as
// [s][q = nt/4][lane][c = nt%4]: value = W[16*nt + (lane&15)][kidx(s, lane)], with
//   first layer:  kidx = 4s + (lane>>4)                 (inputs read from the obs rows)
//   later layers: kidx = 16*(s>>2) + 4*(lane>>4) + (s&3) (inputs = previous accumulators)
__device__ __forceinline__ int kidx(bool first, int s, int lane) {
  return first ? 4 * s + (lane >> 4) : 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
}

__global__ void pack_kernel(int n_out, const float* __restrict__ w1, const float* __restrict__ b1,
                            const float* __restrict__ w2, const float* __restrict__ b2,
                            const float* __restrict__ w3, const float* __restrict__ b3,
                            const float* __restrict__ w4, const float* __restrict__ b4,
                            const float* __restrict__ w5, const float* __restrict__ b5, float* __restrict__ out) {
  const int64_t total = packed_size(n_out);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (e < off_w5()) {
      const float* w;
      int K, N;
      int64_t base;
      bool first = false;
      if (e < off_w2()) { w = w1; K = kIn; N = kH1; base = off_w1(); first = true; }
      else if (e < off_w3()) { w = w2; K = kH1; N = kH2; base = off_w2(); }
      else if (e < off_w4()) { w = w3; K = kH2; N = kH3; base = off_w3(); }
      else { w = w4; K = kH3; N = kH4; base = off_w4(); }
      const int64_t i = e - base;
      const int NQ = N / 64;  // float4 groups of output tiles
      const int c = (int)(i & 3), lane = (int)((i >> 2) & 63);
      const int64_t sq = i >> 8;
      const int q = (int)(sq % NQ), s = (int)(sq / NQ);
      const int nt = 4 * q + c;
      v = w[(int64_t)(16 * nt + (lane & 15)) * K + kidx(first, s, lane)];
    } else if (e < off_b(n_out)) {  // output layer: [a][g][t][r] = W5[a][16t + 4g + r]
      const int64_t i = e - off_w5();
      const int a = (int)(i / kH4), rem = (int)(i % kH4);
      const int g = rem / 64, tr = rem % 64, t = tr / 4, r = tr % 4;
      v = w5[(int64_t)a * kH4 + 16 * t + 4 * g + r];
    } else {
      int64_t i = e - off_b(n_out);
      if (i < kH1) v = b1[i];
      else if ((i -= kH1) < kH2) v = b2[i];
      else if ((i -= kH2) < kH3) v = b3[i];
      else if ((i -= kH3) < kH4) v = b4[i];
      else v = b5[i - kH4];
    }
    out[e] = v;
  }
}

// tanh on the hardware transcendentals (v_exp_f32, v_rcp_f32): sign(x) (1 - t) / (1 + t) with
// t = 2^(-2|x| log2 e); a few ulp from the library tanhf, ~6 instructions instead of ~25.
__device__ __forceinline__ float fast_tanh(float x) {
  const float t = __builtin_amdgcn_exp2f(-2.8853900817779268f * fabsf(x));
  return copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), x);
}

// ---- one MFMA layer: hout = tanh(W . hin + b), all in registers ------------------------------------
// The 4 waves of a workgroup (64 rows) share every weight chunk through LDS: a chunk = CK
// k-steps x (N / OS) outputs, double-buffered.  Each wave loads a quarter of chunk c+1 from L2
// into registers while it runs the MFMAs of chunk c out of LDS, then writes it to the other LDS
// buffer; one workgroup barrier per chunk.  L2 weight traffic is 1/4 of the per-wave streaming
// form.  OS > 1 computes the outputs in OS passes of N / OS (each weight is still read once; the
// inputs stay in registers): OS x fewer live accumulators, which is what keeps the 512-wide layers
// out of scratch.  All loops are unrolled (hin / acc indices static).
#ifndef VPOL_CK
#define VPOL_CK 8
#endif
#ifndef VPOL_OS
#define VPOL_OS 2
#endif
constexpr int kCK = VPOL_CK;                               // k-steps per chunk
constexpr int kOS512 = VPOL_OS;                            // output passes of the 512-wide layers
constexpr int kChunkFloats = kCK * (kH2 / kOS512 > kH1 ? kH2 / kOS512 : kH1) * 4;  // largest chunk (floats)

template <int K4, int NT, int OS>
__device__ __forceinline__ void mfma_layer(const float* __restrict__ wp, const float* __restrict__ bias,
                                           const float (&hin)[K4], float (&hout)[NT * 4], int lane,
                                           float* __restrict__ lds, int wave) {
  static_assert(NT % (4 * OS) == 0, "passes must split whole float4 groups");
  constexpr int NQ = NT / 4;                         // float4 weight groups per k-step (layer)
  constexpr int NTP = NT / OS, NQP = NQ / OS;        // tiles / groups per pass
  constexpr int NCH = (K4 + kCK - 1) / kCK;          // chunks per pass
  constexpr int CH_F4 = kCK * NQP * 64;              // float4 per full chunk
  static_assert(CH_F4 * 4 <= kChunkFloats, "chunk must fit one LDS buffer");
  constexpr int PER_WAVE = (CH_F4 + 3) / 4;          // float4 each wave stages per chunk
  constexpr int PER_LANE = (PER_WAVE + 63) / 64;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(wp);
  f32x4* l4 = reinterpret_cast<f32x4*>(lds);
  const int g = lane >> 4;
  // chunk element e (= (u * NQP + qq) * 64 + l) of chunk c of pass p -> packed float4 index
  auto gidx = [&](int p, int c, int e) {
    const int u = e / (NQP * 64), rest = e - u * (NQP * 64);
    return ((c * kCK + u) * NQ + p * NQP) * 64 + rest;
  };
  auto in_layer = [&](int c, int e) { return c * kCK + e / (NQP * 64) < K4; };
#pragma unroll
  for (int p = 0; p < OS; ++p) {
    f32x4 acc[NTP];
#pragma unroll
    for (int nt = 0; nt < NTP; ++nt) acc[nt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 stage[PER_LANE];
    // chunk 0 -> buffer 0: every load issued before the first LDS write (one wait, not one per load)
#pragma unroll
    for (int j = 0; j < PER_LANE; ++j) {
      const int e = wave * PER_WAVE + j * 64 + lane;
      if (e < (wave + 1) * PER_WAVE && e < CH_F4 && in_layer(0, e)) stage[j] = g4[gidx(p, 0, e)];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < PER_LANE; ++j) {
      const int e = wave * PER_WAVE + j * 64 + lane;
      if (e < (wave + 1) * PER_WAVE && e < CH_F4 && in_layer(0, e)) l4[e] = stage[j];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int buf = c & 1;
      // stage chunk c+1 (L2 -> registers) while chunk c computes
      if (c + 1 < NCH) {
#pragma unroll
        for (int j = 0; j < PER_LANE; ++j) {
          const int e = wave * PER_WAVE + j * 64 + lane;
          if (e < (wave + 1) * PER_WAVE && e < CH_F4 && in_layer(c + 1, e)) stage[j] = g4[gidx(p, c + 1, e)];
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // the next chunk's loads stay ahead of this chunk's MFMAs
      const f32x4* cur = l4 + buf * (kChunkFloats / 4);
      // the weights of k-step u + 1 are read from LDS while k-step u's MFMAs run (two register
      // sets), so the LDS latency hides behind NQP x 4 MFMAs instead of stalling every group
      f32x4 wk[NQP], wn[NQP];
#pragma unroll
      for (int q = 0; q < NQP; ++q) wk[q] = cur[q * 64 + lane];
#pragma unroll
      for (int u = 0; u < kCK; ++u) {
        const int s = c * kCK + u;
        if (s < K4) {
          if (u + 1 < kCK && s + 1 < K4) {
#pragma unroll
            for (int q = 0; q < NQP; ++q) wn[q] = cur[((u + 1) * NQP + q) * 64 + lane];
          }
          // keep those LDS reads ahead of this k-step's MFMAs (the scheduler would sink them to
          // their use); VALU / SALU / transcendental / global-memory work may still move across
          __builtin_amdgcn_sched_barrier(0x416);
#pragma unroll
          for (int q = 0; q < NQP; ++q)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              acc[4 * q + cc] = __builtin_amdgcn_mfma_f32_16x16x4f32(wk[q][cc], hin[s], acc[4 * q + cc], 0, 0, 0);
#pragma unroll
          for (int q = 0; q < NQP; ++q) wk[q] = wn[q];
        }
      }
      if (c + 1 < NCH) {
        f32x4* nxt = l4 + (buf ^ 1) * (kChunkFloats / 4);
#pragma unroll
        for (int j = 0; j < PER_LANE; ++j) {
          const int e = wave * PER_WAVE + j * 64 + lane;
          if (e < (wave + 1) * PER_WAVE && e < CH_F4 && in_layer(c + 1, e)) nxt[e] = stage[j];
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int nt = 0; nt < NTP; ++nt) {
      const int tile = p * NTP + nt;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + 16 * tile + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) hout[4 * tile + r] = fast_tanh(acc[nt][r] + bb[r]);
    }
  }
}

// Full network on this wave's 16 rows; returns the n_out outputs of sample (lane & 15) in every
// lane of its group (the reduction over the 4 lane groups is broadcast).
template <int NOUT>
__device__ __forceinline__ void mlp(const float* __restrict__ packed, const float (&x)[13], float (&out)[NOUT],
                                    int lane, float* lds, int wave) {
  const float* bias = packed + off_b(NOUT);
  float h1[64], h2[128], h3[128], h4[64];
  mfma_layer<13, 16, 1>(packed + off_w1(), bias, x, h1, lane, lds, wave);
  mfma_layer<64, 32, kOS512>(packed + off_w2(), bias + kH1, h1, h2, lane, lds, wave);
  mfma_layer<128, 32, kOS512>(packed + off_w3(), bias + kH1 + kH2, h2, h3, lane, lds, wave);
  mfma_layer<128, 16, 1>(packed + off_w4(), bias + kH1 + kH2 + kH3, h3, h4, lane, lds, wave);
  const int g = lane >> 4;
#pragma unroll
  for (int a = 0; a < NOUT; ++a) {
    const f32x4* w = reinterpret_cast<const f32x4*>(packed + off_w5() + (int64_t)a * kH4 + 64 * g);
    float acc = 0.0f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const f32x4 ww = w[t];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc += ww[r] * h4[4 * t + r];
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    out[a] = acc + bias[kH1 + kH2 + kH3 + kH4 + a];
  }
}

__device__ __forceinline__ void load_rows(const float* __restrict__ obs, int64_t rows, int64_t r0, int lane,
                                          float (&x)[13]) {
  const int64_t row = r0 + (lane & 15);
  const int g = lane >> 4;
#pragma unroll
  for (int s = 0; s < 13; ++s) x[s] = row < rows ? obs[row * kIn + 4 * s + g] : 0.0f;
}

// Philox4x32-10 (same constants as the step kernel); one standard normal pair per call.
__device__ __forceinline__ void normal2(uint64_t seed, uint64_t ctr, uint32_t row, uint32_t blk, float& z0, float& z1) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t c0 = row, c1 = (uint32_t)ctr, c2 = (uint32_t)(ctr >> 32) ^ 0x504f4c00u /* "POL" */, c3 = blk;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  const float u1 = (float)((c0 >> 8) + 1u) * 5.9604645e-08f, u2 = (float)(c1 >> 8) * 5.9604645e-08f;
  const float rad = sqrtf(-2.0f * logf(u1));
  float sn, cs;
  sincosf(6.2831853f * u2, &sn, &cs);
  z0 = rad * cs;
  z1 = rad * sn;
}

struct PolicyArgs {
  int64_t rows;
  const float* obs;
  const float* actor;
  const float* critic;
  const float* logstd;
  const float* action_in;
  float* action_out;
  float* logprob_out;
  float* entropy_out;
  float* value_out;
  float* mean_out;
  uint64_t seed;
  uint64_t counter;
  const int64_t* row_mask;  // critic-only: evaluate / write only rows with row_mask[row] != 0
};

// get_action_and_value (ppo…:157-164): actor mean, Normal(mean, exp(logstd)) sample (or the given
// action), log-prob and entropy summed over action dims, critic value.  CRITIC_ONLY: get_value.
template <int NACT, bool CRITIC_ONLY>
__global__ __launch_bounds__(kWaves * 64) void policy_kernel(PolicyArgs p) {
  __shared__ __attribute__((aligned(16))) float lds[2 * kChunkFloats];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * kWaves + wave) * kRowsPerWave;
  // waves past the last row still take part in the weight staging and barriers
  if (CRITIC_ONLY && p.row_mask) {
    // masked terminal-value pass: a workgroup with no masked row has nothing to do (uniform exit)
    const int64_t wr = (int64_t)blockIdx.x * kWaves * kRowsPerWave + threadIdx.x;
    const bool m = threadIdx.x < kWaves * kRowsPerWave && wr < p.rows && p.row_mask[wr] != 0;
    if (__syncthreads_or(m) == 0) return;
  }
  float x[13];
  load_rows(p.obs, p.rows, r0, lane, x);
  const int64_t row = r0 + (lane & 15);
  const bool writer = (lane >> 4) == 0 && row < p.rows;
  if constexpr (!CRITIC_ONLY) {
    float mean[NACT];
    mlp<NACT>(p.actor, x, mean, lane, lds, wave);
    if (writer) {
      // torch.distributions.Normal: log_prob = -(a-mu)^2/(2 var) - log(scale) - log(sqrt(2 pi));
      // entropy = 0.5 + 0.5 log(2 pi) + log(scale)
      float lp = 0.0f, ent = 0.0f;
#pragma unroll
      for (int a = 0; a < NACT; a += 2) {
        float z0, z1;
        if (!p.action_in) normal2(p.seed, p.counter, (uint32_t)row, (uint32_t)a, z0, z1);
#pragma unroll
        for (int h = 0; h < 2 && a + h < NACT; ++h) {
          const float scale = expf(p.logstd[a + h]);
          const float act = p.action_in ? p.action_in[row * NACT + a + h] : mean[a + h] + scale * (h ? z1 : z0);
          const float d = act - mean[a + h];
          const float log_scale = logf(scale);
          lp += -(d * d) / (2.0f * (scale * scale)) - log_scale - 0.91893853320467274f;
          ent += 0.5f + 0.91893853320467274f + log_scale;
          if (p.action_out) p.action_out[row * NACT + a + h] = act;
          if (p.mean_out) p.mean_out[row * NACT + a + h] = mean[a + h];
        }
      }
      if (p.logprob_out) p.logprob_out[row] = lp;
      if (p.entropy_out) p.entropy_out[row] = ent;
    }
  }
  float v[1];
  mlp<1>(p.critic, x, v, lane, lds, wave);
  const bool masked_out = CRITIC_ONLY && p.row_mask && writer && p.row_mask[row] == 0;
  if (writer && !masked_out && p.value_out) p.value_out[row] = v[0];
}

}  // namespace vpol

extern "C" {

int64_t vss_mlp_packed_size(int32_t n_out) {
  return (n_out >= 1 && n_out <= 8) ? vpol::packed_size(n_out) : -1;
}

int vss_mlp_pack(void* stream, int32_t n_out, const float* const* weights, const float* const* biases, float* packed) {
  if (n_out < 1 || n_out > 8 || !weights || !biases || !packed || (reinterpret_cast<uintptr_t>(packed) & 15))
    return VSS_E_ARG;
  for (int i = 0; i < 5; ++i)
    if (!weights[i] || !biases[i]) return VSS_E_ARG;
  hipLaunchKernelGGL(vpol::pack_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, n_out, weights[0], biases[0],
                     weights[1], biases[1], weights[2], biases[2], weights[3], biases[3], weights[4], biases[4], packed);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_policy_forward(void* stream, int64_t rows, int32_t n_act, const float* obs, const float* actor_packed,
                       const float* logstd, const float* critic_packed, uint64_t seed, uint64_t counter,
                       const float* action_in, float* action_out, float* logprob_out, float* entropy_out,
                       float* value_out, float* mean_out) {
  return vss_value_forward_masked(stream, rows, n_act, obs, actor_packed, logstd, critic_packed, seed, counter,
                                  action_in, action_out, logprob_out, entropy_out, value_out, mean_out, nullptr);
}

int vss_value_forward_masked(void* stream, int64_t rows, int32_t n_act, const float* obs, const float* actor_packed,
                             const float* logstd, const float* critic_packed, uint64_t seed, uint64_t counter,
                             const float* action_in, float* action_out, float* logprob_out, float* entropy_out,
                             float* value_out, float* mean_out, const int64_t* row_mask) {
  // packed weights are read as float4 (16-B aligned), the mask as int64
  auto misaligned = [](const void* ptr, uintptr_t al) { return (reinterpret_cast<uintptr_t>(ptr) & (al - 1)) != 0; };
  if (rows < 0 || !obs || !critic_packed || misaligned(critic_packed, 16) || misaligned(actor_packed, 16) ||
      misaligned(row_mask, 8))
    return VSS_E_ARG;
  const bool critic_only = actor_packed == nullptr;
  if (!critic_only && (!logstd || !(n_act == 2 || n_act == 6))) return VSS_E_ARG;
  if (row_mask && !critic_only) return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  vpol::PolicyArgs a{rows, obs, actor_packed, critic_packed, logstd, action_in, action_out, logprob_out,
                     entropy_out, value_out, mean_out, seed, counter, row_mask};
  const int64_t waves = (rows + vpol::kRowsPerWave - 1) / vpol::kRowsPerWave;
  const dim3 grid((unsigned)((waves + vpol::kWaves - 1) / vpol::kWaves)), block(vpol::kWaves * 64);
  hipStream_t s = (hipStream_t)stream;
  if (critic_only) hipLaunchKernelGGL((vpol::policy_kernel<2, true>), grid, block, 0, s, a);
  else if (n_act == 2) hipLaunchKernelGGL((vpol::policy_kernel<2, false>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((vpol::policy_kernel<6, false>), grid, block, 0, s, a);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
