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
// registers from the first layer to the last (no LDS, no HBM round trips).  Bias + tanh, the tiny
// output layer (VALU dot products + cross-lane reduction), Gaussian sampling (Philox), log-prob and
// entropy are fused into the epilogue.
//
// Weights: one flat STREAM per network.  Every hidden layer is cut into passes of 16 output tiles
// (256 features: the 512-wide layers take two passes, so only 64 accumulators are live), and a
// pass's k-steps are uniform blocks of 16 tiles x 64 lanes x 4 k = 1,024 floats (4 KB):
//   layer 1: 16 k-steps (K = 52 padded to 64; k-steps 13-15 hold zeros and are never multiplied)
//   layer 2: 2 passes x 64 k-steps, layer 3: 2 x 128, layer 4: 1 x 128          = 528 k-steps
// The 4 waves of a workgroup (64 rows) share the stream through a double-buffered LDS ring of
// chunks of kCK = 8 k-steps (32 KB): during chunk g every wave loads a quarter of chunk g + 1 into
// registers (issued before chunk g's MFMAs, so the L2 / Infinity-Cache latency hides behind them),
// writes it to the other buffer before chunk g's last k-step, and one workgroup barrier per chunk
// publishes it.  The stream runs on across pass and layer boundaries, so no pass starts with an
// exposed load; each pass's bias + tanh epilogue is drained between the next pass's MFMAs.  (Round 2's form restarted the staging at every pass with one serial
// load -> wait -> LDS write per float4, and the compiler sank part of each chunk's prefetch behind
// its MFMAs: 0.60 of the MFMA peak.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_policy.hip targets gfx950 (CDNA4) only"
#endif

namespace vpol {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIn = 52, kH1 = 256, kH2 = 512, kH3 = 512, kH4 = 256;
constexpr int kWaves = 4;          // waves per workgroup (64 rows per workgroup), one per SIMD
constexpr int64_t kBothMaxWorkgroups = 128;  // up to 8,192 rows: actor and critic in one launch
constexpr int kRowsPerWave = 16;
constexpr int kTiles = 16;                         // output tiles of one pass (256 features)
constexpr int kStepFloats = kTiles * 16 * 4;       // one pass's weights for one k-step: 1,024 floats
constexpr int kCK = 8;                             // k-steps per chunk
constexpr int kChunkF4 = kCK * kStepFloats / 4;    // float4 per chunk (2,048 = 32 KB)
constexpr int kStepsL1 = 16, kStepsL2 = 64, kStepsL3 = 128, kStepsL4 = 128;
constexpr int kUsedStepsL1 = kIn / 4;              // 13
constexpr int kStreamSteps = kStepsL1 + 2 * kStepsL2 + 2 * kStepsL3 + kStepsL4;  // 528
constexpr int kNetChunks = kStreamSteps / kCK;     // 66
static_assert(kStepsL1 % kCK == 0 && kStepsL2 % kCK == 0 && kStepsL3 % kCK == 0, "passes must be whole chunks");
constexpr int kStageF4 = kChunkF4 / (kWaves * 64);  // float4 each lane stages per chunk (8)
// first chunk of each pass within a network's stream
constexpr int kG1 = 0, kG2a = kStepsL1 / kCK, kG2b = kG2a + kStepsL2 / kCK, kG3a = kG2b + kStepsL2 / kCK,
              kG3b = kG3a + kStepsL3 / kCK, kG4 = kG3b + kStepsL3 / kCK;
static_assert(kG4 + kStepsL4 / kCK == kNetChunks, "stream layout");

// packed-buffer offsets (floats) of one network with n_out outputs
__host__ __device__ constexpr int64_t off_w5() { return (int64_t)kStreamSteps * kStepFloats; }
__host__ __device__ constexpr int64_t off_b(int n_out) { return off_w5() + (int64_t)n_out * kH4; }
__host__ __device__ constexpr int64_t packed_size(int n_out) {
  return off_b(n_out) + kH1 + kH2 + kH3 + kH4 + n_out;
}
// the packed tail past the stream (output-layer weights, then every bias): staged into LDS once per
// workgroup, so the epilogues read it with ds_read (lgkmcnt) -- a global load there would wait, by
// vmcnt's in-order count, for the next chunk's staging loads issued before it
__host__ __device__ constexpr int tail_floats(int n_out) { return (int)(packed_size(n_out) - off_w5()); }

// ---- packing ---------------------------------------------------------------------------------------
// Stream k-step block (layer, pass p, k-step s): [q = 0..3][lane][c = 0..3], value
// W[16 nt + (lane & 15)][kidx(s, lane)] with nt = 16 p + 4 q + c, and
//   layer 1:      kidx = 4 s + (lane >> 4)                    (inputs read from the obs rows)
//   later layers: kidx = 16 (s >> 2) + 4 (lane >> 4) + (s & 3) (inputs = previous accumulators)
// (zero for kidx >= K: layer 1's padding).
__global__ void pack_kernel(int n_out, const float* __restrict__ w1, const float* __restrict__ b1,
                            const float* __restrict__ w2, const float* __restrict__ b2,
                            const float* __restrict__ w3, const float* __restrict__ b3,
                            const float* __restrict__ w4, const float* __restrict__ b4,
                            const float* __restrict__ w5, const float* __restrict__ b5, float* __restrict__ out) {
  const int64_t total = packed_size(n_out);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (e < off_w5()) {
      int blk = (int)(e / kStepFloats);
      const int i = (int)(e % kStepFloats);
      const int c = i & 3, lane = (i >> 2) & 63, q = i >> 8;
      const float* w;
      int K, s, p = 0;
      bool first = false;
      if (blk < kStepsL1) { w = w1; K = kIn; s = blk; first = true; }
      else if ((blk -= kStepsL1) < 2 * kStepsL2) { w = w2; K = kH1; p = blk / kStepsL2; s = blk % kStepsL2; }
      else if ((blk -= 2 * kStepsL2) < 2 * kStepsL3) { w = w3; K = kH2; p = blk / kStepsL3; s = blk % kStepsL3; }
      else { blk -= 2 * kStepsL3; w = w4; K = kH3; s = blk; }
      const int nt = kTiles * p + 4 * q + c;
      const int k = first ? 4 * s + (lane >> 4) : 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
      v = k < K ? w[(int64_t)(16 * nt + (lane & 15)) * K + k] : 0.0f;
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

// ---- the weight stream ------------------------------------------------------------------------------
// Chunk g of a launch's stream (one network's kNetChunks chunks).  Every chunk index below is a
// compile-time constant once the pass loops are unrolled.
struct Stream {
  const f32x4* net;
  f32x4* lds;  // two chunk buffers
  int wave, lane, last;
  f32x4 stage[kStageF4];
  f32x4 first[4];  // the weights of the current chunk's first k-step (read before it starts)

  __device__ __forceinline__ void load(int g) {
    const f32x4* src = net + (int64_t)g * kChunkF4;
#pragma unroll
    for (int j = 0; j < kStageF4; ++j) stage[j] = src[(wave * kStageF4 + j) * 64 + lane];
  }
  __device__ __forceinline__ void store(int g) {
    f32x4* dst = lds + (g & 1) * kChunkF4;
#pragma unroll
    for (int j = 0; j < kStageF4; ++j) dst[(wave * kStageF4 + j) * 64 + lane] = stage[j];
  }
};

// One pass of NSTEPS k-steps (the first NUSED multiplied) into kTiles output tiles, out of the
// stream's chunks g0, g0 + 1, ...: hin holds the layer's B operands (one per k-step); the raw
// accumulators are left in acc.  Their bias + tanh epilogue is DEFERRED into the next pass, which
// drains it tile by tile between its own MFMAs (one wave per SIMD: nothing else would hide that VALU
// work): with DRAIN, pend holds the previous pass's accumulators and tile j becomes
// pdst[4 (DT0 + j) + r] = tanh(pend[j][r] + pbias[16 (DT0 + j) + 4 (lane >> 4) + r]) -- tile 0 before
// the first k-step, tile j after k-step j - 1.  When pdst is this pass's own hin (the previous
// layer's last pass), k-step s reads tile s >> 2, which has been drained by then.
__device__ __forceinline__ void drain_tile(const f32x4& pend, const float* pbias, float* dst, int grp) {
  const f32x4 bb = *reinterpret_cast<const f32x4*>(pbias + 4 * grp);  // LDS
#pragma unroll
  for (int r = 0; r < 4; ++r) dst[r] = fast_tanh(pend[r] + bb[r]);
}

template <int NSTEPS, int NUSED, bool DRAIN, int DT0, int KIN, int NDST>
__device__ __forceinline__ void mfma_pass(Stream& st, int g0, const float (&hin)[KIN], f32x4 (&acc)[kTiles],
                                          const f32x4 (&pend)[kTiles], const float* pbias, float (&pdst)[NDST]) {
  static_assert(NSTEPS % kCK == 0 && NUSED <= NSTEPS && NUSED <= KIN, "pass shape");
  static_assert(!DRAIN || (NUSED >= kTiles && 4 * (DT0 + kTiles) <= NDST), "drain shape");
  constexpr int NCH = NSTEPS / kCK;
  const int lane = st.lane, grp = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < kTiles; ++nt) acc[nt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  if constexpr (DRAIN) drain_tile(pend[0], pbias + 16 * DT0, pdst + 4 * DT0, grp);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int g = g0 + c;
    const bool more = g + 1 <= st.last;
    const int uc = NUSED - c * kCK < kCK ? NUSED - c * kCK : kCK;  // k-steps of this chunk multiplied
    if (more) st.load(g + 1);  // the next chunk (possibly the next pass's / network's), L2 -> registers
    __builtin_amdgcn_sched_barrier(0);  // keep those loads ahead of this chunk's MFMAs
    const f32x4* cur = st.lds + (g & 1) * kChunkF4;
    // the weights of k-step u + 1 are read from LDS while k-step u's MFMAs run (two register sets)
    f32x4 wk[4], wn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) wk[q] = st.first[q];
#pragma unroll
    for (int u = 0; u < kCK; ++u) {
      const int s = c * kCK + u;
      if (u < uc) {
        if (u + 1 < uc) {
#pragma unroll
          for (int q = 0; q < 4; ++q) wn[q] = cur[((u + 1) * 4 + q) * 64 + lane];
        } else if (more) {
          // Before the chunk's last k-step (whose weights are in registers): publish chunk g + 1 --
          // its buffer was last read before the previous chunk's barrier -- and read its first k-step
          // while this k-step's MFMAs run, so the next chunk starts without an LDS round trip.  Every
          // LDS read of chunk g has completed (the barrier's fence), so the buffer is free after it.
          st.store(g + 1);
          __syncthreads();
          const f32x4* nxt = st.lds + ((g + 1) & 1) * kChunkF4;
#pragma unroll
          for (int q = 0; q < 4; ++q) st.first[q] = nxt[q * 64 + lane];
        }
        // keep those LDS reads ahead of this k-step's MFMAs (the scheduler would sink them to their
        // use); VALU / SALU / transcendental / global-memory work may still move across
        __builtin_amdgcn_sched_barrier(0x416);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
            acc[4 * q + cc] = __builtin_amdgcn_mfma_f32_16x16x4f32(wk[q][cc], hin[s], acc[4 * q + cc], 0, 0, 0);
        if constexpr (DRAIN) {
          if (s + 1 < kTiles) drain_tile(pend[s + 1], pbias + 16 * (DT0 + s + 1), pdst + 4 * (DT0 + s + 1), grp);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) wk[q] = wn[q];
      }
    }
  }
}

// One network on this wave's 16 rows, its stream chunks starting at g0, its packed tail (output
// weights + biases, tail_floats) in LDS at `tail`; returns the NOUT outputs of sample (lane & 15) in
// every lane of its group (the reduction over the 4 lane groups is broadcast).  Passes alternate
// between two accumulator sets: each pass drains the previous one's epilogue.
template <int NOUT>
__device__ __forceinline__ void mlp(Stream& st, int g0, const float* tail, const float (&x)[16], float (&out)[NOUT]) {
  const float* bias = tail + NOUT * kH4;
  const float *b1 = bias, *b2 = b1 + kH1, *b3 = b2 + kH2, *b4 = b3 + kH3;
  float h1[64], h2[128], h3[128], h4[64];
  f32x4 A[kTiles], B[kTiles];
  mfma_pass<kStepsL1, kUsedStepsL1, false, 0>(st, g0 + kG1, x, A, B, b1, h1);        // B unused
  mfma_pass<kStepsL2, kStepsL2, true, 0>(st, g0 + kG2a, h1, B, A, b1, h1);           // drains h1
  mfma_pass<kStepsL2, kStepsL2, true, 0>(st, g0 + kG2b, h1, A, B, b2, h2);           // h2 tiles 0-15
  mfma_pass<kStepsL3, kStepsL3, true, kTiles>(st, g0 + kG3a, h2, B, A, b2, h2);      // h2 tiles 16-31
  mfma_pass<kStepsL3, kStepsL3, true, 0>(st, g0 + kG3b, h2, A, B, b3, h3);           // h3 tiles 0-15
  mfma_pass<kStepsL4, kStepsL4, true, kTiles>(st, g0 + kG4, h3, B, A, b3, h3);       // h3 tiles 16-31
  const int g = st.lane >> 4;
#pragma unroll
  for (int nt = 0; nt < kTiles; ++nt) drain_tile(B[nt], b4 + 16 * nt, h4 + 4 * nt, g);  // the last pass: eager
#pragma unroll
  for (int a = 0; a < NOUT; ++a) {
    const f32x4* w = reinterpret_cast<const f32x4*>(tail + a * kH4 + 64 * g);
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

// the first layer's B operands: x[s] = obs[row][4 s + (lane >> 4)] (s < 13; the padding k-steps 0)
__device__ __forceinline__ void load_rows(const float* __restrict__ obs, int64_t rows, int64_t r0, int lane,
                                          float (&x)[16]) {
  const int64_t row = r0 + (lane & 15);
  const int g = lane >> 4;
#pragma unroll
  for (int s = 0; s < 16; ++s) x[s] = (s < kUsedStepsL1 && row < rows) ? obs[row * kIn + 4 * s + g] : 0.0f;
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

// get_action_and_value's tail (ppo…:157-164) for one row from its actor mean: Normal(mean,
// exp(logstd)) sample (Philox, or the given action), log-prob and entropy summed over the action
// dims.  torch.distributions.Normal: log_prob = -(a-mu)^2/(2 var) - log(scale) - log(sqrt(2 pi));
// entropy = 0.5 + 0.5 log(2 pi) + log(scale).  Shared by the fused kernel and vss_policy_sample, so
// both draw the same actions from the same (seed, counter, row).
template <int NACT>
__device__ __forceinline__ void actor_tail(const float (&mean)[NACT], int64_t row, const float* logstd, uint64_t seed,
                                           uint64_t counter, const float* action_in, float* action_out,
                                           float* logprob_out, float* entropy_out, float* mean_out) {
  float lp = 0.0f, ent = 0.0f;
#pragma unroll
  for (int a = 0; a < NACT; a += 2) {
    float z0, z1;
    if (!action_in) normal2(seed, counter, (uint32_t)row, (uint32_t)a, z0, z1);
#pragma unroll
    for (int h = 0; h < 2 && a + h < NACT; ++h) {
      const float scale = expf(logstd[a + h]);
      const float act = action_in ? action_in[row * NACT + a + h] : mean[a + h] + scale * (h ? z1 : z0);
      const float d = act - mean[a + h];
      const float log_scale = logf(scale);
      lp += -(d * d) / (2.0f * (scale * scale)) - log_scale - 0.91893853320467274f;
      ent += 0.5f + 0.91893853320467274f + log_scale;
      if (action_out) action_out[row * NACT + a + h] = act;
      if (mean_out) mean_out[row * NACT + a + h] = mean[a + h];
    }
  }
  if (logprob_out) logprob_out[row] = lp;
  if (entropy_out) entropy_out[row] = ent;
}

// the same tail over rows whose actor means were computed elsewhere (the rollout's GEMM-chain path)
template <int NACT>
__global__ __launch_bounds__(256) void sample_kernel(int64_t rows, const float* __restrict__ mean, const float* logstd,
                                                     uint64_t seed, uint64_t counter, const float* action_in,
                                                     float* action_out, float* logprob_out, float* entropy_out) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= rows) return;
  float m[NACT];
#pragma unroll
  for (int a = 0; a < NACT; ++a) m[a] = mean[row * NACT + a];
  actor_tail<NACT>(m, row, logstd, seed, counter, action_in, action_out, logprob_out, entropy_out, nullptr);
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

// get_action_and_value (ppo…:157-164) as two launches over the same rows, one network each:
// ACTOR = true: actor mean, Normal(mean, exp(logstd)) sample (or the given action), log-prob and
// entropy summed over action dims; ACTOR = false: the critic's value (Agent.get_value; with row_mask,
// only the masked rows).  One network per launch keeps the weight stream that the concurrently running
// workgroups read at 2.1 MB, inside one XCD's 4 MB L2 (actor + critic in one launch stream 4.3 MB and
// measured 2.6 % slower: profiles/r03f_policy_bench.log).
// One network (ACTOR: the actor and the sampling tail; else the critic) on workgroup `blk`'s rows.
template <int NACT, bool ACTOR>
__device__ __forceinline__ void policy_body(const PolicyArgs& p, int64_t blk, f32x4* lds, float* tails) {
  constexpr int NOUT = ACTOR ? NACT : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (blk * kWaves + wave) * kRowsPerWave;
  // waves past the last row still take part in the weight staging and barriers
  if (!ACTOR && p.row_mask) {
    // masked terminal-value pass: a workgroup with no masked row has nothing to do (uniform exit)
    const int64_t wr = blk * kWaves * kRowsPerWave + threadIdx.x;
    const bool m = threadIdx.x < kWaves * kRowsPerWave && wr < p.rows && p.row_mask[wr] != 0;
    if (__syncthreads_or(m) == 0) return;
  }
  const float* net = ACTOR ? p.actor : p.critic;
  Stream st;
  st.net = reinterpret_cast<const f32x4*>(net);
  st.lds = lds;
  st.wave = wave;
  st.lane = lane;
  st.last = kNetChunks - 1;
  st.load(0);  // the stream's first chunk
  float x[16];
  load_rows(p.obs, p.rows, r0, lane, x);
  for (int i = threadIdx.x; i < tail_floats(NOUT); i += kWaves * 64) tails[i] = net[off_w5() + i];
  st.store(0);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) st.first[q] = lds[q * 64 + lane];
  const int64_t row = r0 + (lane & 15);
  const bool writer = (lane >> 4) == 0 && row < p.rows;
  float out[NOUT];
  mlp<NOUT>(st, 0, tails, x, out);
  if constexpr (ACTOR) {
    if (writer)
      actor_tail<NACT>(out, row, p.logstd, p.seed, p.counter, p.action_in, p.action_out, p.logprob_out, p.entropy_out,
                       p.mean_out);
  } else {
    const bool masked_out = p.row_mask && writer && p.row_mask[row] == 0;
    if (writer && !masked_out && p.value_out) p.value_out[row] = out[0];
  }
}

template <int NACT, bool ACTOR>
__global__ __launch_bounds__(kWaves * 64) void policy_kernel(PolicyArgs p) {
  __shared__ __attribute__((aligned(16))) f32x4 lds[2 * kChunkF4];
  __shared__ __attribute__((aligned(16))) float tails[tail_floats(ACTOR ? NACT : 1)];
  policy_body<NACT, ACTOR>(p, blockIdx.x, lds, tails);
}

// Actor and critic in ONE launch (the first half of the grid runs the actor, the second the critic):
// for small batches (the reference's 4,095 envs: 64 workgroups per network) the two networks then
// run side by side on 128 CUs instead of one after the other, each launch latency-bound on its
// 66-chunk weight stream.  At 65,536 rows two launches measured 2.6 % faster (the concurrently
// read weight stream stays in one XCD's L2), and the rollout uses the GEMM chain there anyway.
template <int NACT>
__global__ __launch_bounds__(kWaves * 64) void policy_kernel_both(PolicyArgs p) {
  __shared__ __attribute__((aligned(16))) f32x4 lds[2 * kChunkF4];
  __shared__ __attribute__((aligned(16))) float tails[tail_floats(NACT)];
  const int64_t half = gridDim.x / 2;
  if ((int64_t)blockIdx.x < half) policy_body<NACT, true>(p, blockIdx.x, lds, tails);
  else policy_body<NACT, false>(p, (int64_t)blockIdx.x - half, lds, tails);
}

// ---- small batches: each pass's 16 output tiles split over the workgroup's 4 waves ---------------------
// Up to kBothMaxWorkgroups x 64 rows (the reference's 4,095 envs) the kernels above run one wave per 16
// rows, so only rows / 16 of the 1,024 SIMDs work and each of them multiplies every weight: 4,095 rows
// keep 512 SIMDs busy for 2,100 MFMAs x 4 per network.  Here a workgroup takes ONE 16-row group and
// its 4 waves split every pass's 16 tiles (wave w: tiles 4 w .. 4 w + 3 of each pass, i.e. float4 q = w
// of each k-step block, read straight from L2 -- no staging ring), so each wave runs a quarter of the
// MFMAs and the row groups x 4 waves fill the chip.  A layer's activations go through LDS: every wave
// writes its tiles in the B-operand layout h[nt][lane] (lane: row lane & 15, features 16 nt + 4
// (lane >> 4) + 0..3) and, after one barrier, reads all of them back into registers for the next
// layer (two buffers, so a wave's writes never meet another wave's reads of the same buffer).  The
// arithmetic per output -- the k order, the MFMA chain, bias + tanh, the output layer, the sampling tail
// -- is that of policy_kernel.
// up to 256 row groups (4,096 rows): actor + critic = 512 workgroups, one pass of two per CU.  Against
// policy_kernel_both, same bits: 4,095 rows 110 vs 156 us, 1 row 58 vs 149 us; at 8,192 rows (two passes)
// 206 vs 157 us, so larger batches keep the kernels above (profiles/r04_policy_split_ab.log)
constexpr int64_t kSplitMaxGroups = 256;
constexpr int kSplitPrefetch = 4;                   // k-steps of weights in flight per wave
constexpr int kSplitBuf = (kH2 / 16) * 64;          // f32x4 per activation buffer (512 features: 32 KB)

template <int S, int NUSED, int NP, int KIN>
__device__ __forceinline__ void split_layer(const f32x4* __restrict__ blocks, const float (&hin)[KIN], f32x4 (&acc)[NP][4],
                                            int wave, int lane) {
  // blocks: the layer's first k-step block; pass p, k-step s at block p S + s; this wave's float4 is q = wave
  const f32x4* src = blocks + wave * 64 + lane;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[p][c] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  f32x4 w[kSplitPrefetch][NP];
#pragma unroll
  for (int s = 0; s < kSplitPrefetch && s < NUSED; ++s)
#pragma unroll
    for (int p = 0; p < NP; ++p) w[s][p] = src[(int64_t)(p * S + s) * (kStepFloats / 4)];
#pragma unroll
  for (int s = 0; s < NUSED; ++s) {
    f32x4 cur[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) cur[p] = w[s % kSplitPrefetch][p];
    if (s + kSplitPrefetch < NUSED) {
#pragma unroll
      for (int p = 0; p < NP; ++p)
        w[s % kSplitPrefetch][p] = src[(int64_t)(p * S + s + kSplitPrefetch) * (kStepFloats / 4)];
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[p][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur[p][c], hin[s], acc[p][c], 0, 0, 0);
  }
}

// bias + tanh of this wave's tiles (pass p, tile 4 wave + c) into the activation buffer, B-operand layout
template <int NP>
__device__ __forceinline__ void split_store(const f32x4 (&acc)[NP][4], const float* bias, f32x4* buf, int wave, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int nt = kTiles * p + 4 * wave + c;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);  // LDS
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fast_tanh(acc[p][c][r] + bb[r]);
      buf[nt * 64 + lane] = v;
    }
}

// all NT tiles of a layer's output back into the B operands of the next layer's k-steps
template <int NT>
__device__ __forceinline__ void split_load(const f32x4* buf, int lane, float (&h)[4 * NT]) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const f32x4 v = buf[nt * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) h[4 * nt + r] = v[r];
  }
}

template <int NACT, bool ACTOR>
__device__ __forceinline__ void split_body(const PolicyArgs& p, int64_t grp, f32x4* hb, float* tails) {
  constexpr int NOUT = ACTOR ? NACT : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* net = ACTOR ? p.actor : p.critic;
  const f32x4* stream = reinterpret_cast<const f32x4*>(net);
  const int64_t r0 = grp * kRowsPerWave;
  for (int i = threadIdx.x; i < tail_floats(NOUT); i += kWaves * 64) tails[i] = net[off_w5() + i];
  float x[16];
  load_rows(p.obs, p.rows, r0, lane, x);
  __syncthreads();
  const float* bias = tails + NOUT * kH4;
  const float *b1 = bias, *b2 = b1 + kH1, *b3 = b2 + kH2, *b4 = b3 + kH3;
  f32x4* buf0 = hb;
  f32x4* buf1 = hb + kSplitBuf;
  {
    f32x4 acc[1][4];
    split_layer<kStepsL1, kUsedStepsL1, 1, 16>(stream, x, acc, wave, lane);
    split_store<1>(acc, b1, buf0, wave, lane);
  }
  __syncthreads();
  {
    float h[kH1 / 4];
    split_load<kH1 / 16>(buf0, lane, h);
    f32x4 acc[2][4];
    split_layer<kStepsL2, kStepsL2, 2, kH1 / 4>(stream + (int64_t)kStepsL1 * (kStepFloats / 4), h, acc, wave, lane);
    split_store<2>(acc, b2, buf1, wave, lane);
  }
  __syncthreads();
  {
    float h[kH2 / 4];
    split_load<kH2 / 16>(buf1, lane, h);
    f32x4 acc[2][4];
    split_layer<kStepsL3, kStepsL3, 2, kH2 / 4>(stream + (int64_t)(kStepsL1 + 2 * kStepsL2) * (kStepFloats / 4), h, acc,
                                                wave, lane);
    split_store<2>(acc, b3, buf0, wave, lane);
  }
  __syncthreads();
  {
    float h[kH3 / 4];
    split_load<kH3 / 16>(buf0, lane, h);
    f32x4 acc[1][4];
    split_layer<kStepsL4, kStepsL4, 1, kH3 / 4>(
        stream + (int64_t)(kStepsL1 + 2 * kStepsL2 + 2 * kStepsL3) * (kStepFloats / 4), h, acc, wave, lane);
    split_store<1>(acc, b4, buf1, wave, lane);
  }
  __syncthreads();
  if (wave != 0) return;
  // the output layer and the tail as mlp() / policy_body do, on wave 0
  float h4[kH4 / 4];
  split_load<kH4 / 16>(buf1, lane, h4);
  const int g = lane >> 4;
  float out[NOUT];
#pragma unroll
  for (int a = 0; a < NOUT; ++a) {
    const f32x4* w = reinterpret_cast<const f32x4*>(tails + a * kH4 + 64 * g);
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
  const int64_t row = r0 + (lane & 15);
  const bool writer = g == 0 && row < p.rows;
  if constexpr (ACTOR) {
    if (writer)
      actor_tail<NACT>(out, row, p.logstd, p.seed, p.counter, p.action_in, p.action_out, p.logprob_out, p.entropy_out,
                       p.mean_out);
  } else {
    if (writer && p.value_out) p.value_out[row] = out[0];
  }
}

// actor and critic of every 16-row group in one launch: blocks [0, groups) the actor, [groups, 2 groups)
// the critic; 2 workgroups per CU (LDS: two 32-KB activation buffers + the packed tail)
template <int NACT>
__global__ __launch_bounds__(kWaves * 64, 2) void policy_split_kernel(PolicyArgs p) {
  __shared__ __attribute__((aligned(16))) f32x4 hb[2 * kSplitBuf];
  __shared__ __attribute__((aligned(16))) float tails[tail_floats(NACT)];
  const int64_t groups = gridDim.x / 2;
  if ((int64_t)blockIdx.x < groups) split_body<NACT, true>(p, blockIdx.x, hb, tails);
  else split_body<NACT, false>(p, (int64_t)blockIdx.x - groups, hb, tails);
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
  const int64_t wgs = (waves + vpol::kWaves - 1) / vpol::kWaves;
  const dim3 grid((unsigned)wgs), block(vpol::kWaves * 64);
  hipStream_t s = (hipStream_t)stream;
  if (!critic_only && waves <= vpol::kSplitMaxGroups) {
    // small batch: both networks in one launch, one workgroup per 16-row group, tiles split over its waves
    const dim3 grid2((unsigned)(2 * waves));
    if (n_act == 2) hipLaunchKernelGGL((vpol::policy_split_kernel<2>), grid2, block, 0, s, a);
    else hipLaunchKernelGGL((vpol::policy_split_kernel<6>), grid2, block, 0, s, a);
    return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
  }
  if (!critic_only && wgs <= vpol::kBothMaxWorkgroups) {  // both networks in one launch
    const dim3 grid2((unsigned)(2 * wgs));
    if (n_act == 2) hipLaunchKernelGGL((vpol::policy_kernel_both<2>), grid2, block, 0, s, a);
    else hipLaunchKernelGGL((vpol::policy_kernel_both<6>), grid2, block, 0, s, a);
    return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
  }
  if (!critic_only) {
    if (n_act == 2) hipLaunchKernelGGL((vpol::policy_kernel<2, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((vpol::policy_kernel<6, true>), grid, block, 0, s, a);
  }
  hipLaunchKernelGGL((vpol::policy_kernel<1, false>), grid, block, 0, s, a);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_policy_sample(void* stream, int64_t rows, int32_t n_act, const float* mean, const float* logstd, uint64_t seed,
                      uint64_t counter, const float* action_in, float* action_out, float* logprob_out,
                      float* entropy_out) {
  if (rows < 0 || !mean || !logstd || !(n_act == 2 || n_act == 6)) return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const dim3 grid((unsigned)((rows + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (n_act == 2)
    hipLaunchKernelGGL(vpol::sample_kernel<2>, grid, block, 0, s, rows, mean, logstd, seed, counter, action_in,
                       action_out, logprob_out, entropy_out);
  else
    hipLaunchKernelGGL(vpol::sample_kernel<6>, grid, block, 0, s, rows, mean, logstd, seed, counter, action_in,
                       action_out, logprob_out, entropy_out);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
