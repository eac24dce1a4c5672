// vss_update.hip — PPO-update helpers on gfx950 (ppo_continuous_action_isaacgym.py:306-353).
//
// 1. vss_tanh_grad_bias: the backward of a hidden tanh layer as one memory-bound pass.
//    The update back-propagates through the Agent's tanh MLPs (ppo…:104-125).  For each hidden
//    layer torch issues two memory-bound passes over the (rows x cols) gradient: tanh_backward
//    (gz = gy * (1 - y^2): read gy, y, write gz) and the bias gradient (db = sum over rows of gz:
//    read gz again).  This kernel does both in one pass: every workgroup owns a fixed set of row
//    tiles, writes gz and one row of column sums; the caller reduces the (workgroups x cols)
//    partial sums (a few MB) to db.  The tile assignment and the order of the sums are fixed, so
//    db is deterministic.  HBM bytes per element: 12 (gy, y read, gz write) instead of 16.
// 2. vss_linear_tanh / vss_linear_tanh_backward: the hidden layers' GEMMs on the fp32 matrix cores
//    with the elementwise work in their epilogues (below).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vss.h"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_update.hip targets gfx950 (CDNA4) only"
#endif

namespace vupd {

constexpr int kThreads = 256;
constexpr int kU = 8;                  // rows per lane in flight (2 x kU 16-B loads before the first use)
constexpr int kWavesPerSimd = 4;       // register budget: all 2 kU loads of a lane in flight
constexpr int64_t kMaxBlocks = 2048;   // the partial sums are (blocks x cols)

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld(const float4* p) { return *p; }

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
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, kWavesPerSimd))) void tanh_grad_bias_kernel(
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

// ---- the hidden layers' GEMMs with fused epilogues, fp32 matrix cores --------------------------------
// out = A B^T with A (rows, K) row-major and B (n, K) row-major (nn.Linear's weight layout), both
// K-contiguous, and one of two epilogues:
//   EPI_TANH   (forward, ppo…:104-111 nn.Linear then nn.Tanh):  out = tanh(acc + bias)
//              — one launch instead of hipBLASLt's addmm plus torch's tanh pass (which re-reads and
//              re-writes the whole activation);
//   EPI_DTANH  (backward through the NEXT layer and this layer's tanh): with A = the next layer's
//              pre-activation gradient and B = the next layer's weight transposed,
//              out = acc * (1 - y^2) (y = this layer's tanh output) and per-block column sums of out
//              (the bias gradient) — instead of addmm's gy write plus vss_tanh_grad_bias's pass.
// Block tile 128 x 128, K tiles of 32 through a double-buffered LDS image (register staging: the
// next K tile's global loads are in flight during this K tile's MFMAs; one barrier per K tile);
// 4 waves as 2 x 2, each a 64 x 64 output = 2 x 2 tiles of v_mfma_f32_32x32x2_f32 (exact fp32 FMA
// chains).  k order: lane half h of a 32x32x2 step takes k = 16h + 4q + s of the 32-wide tile
// (q = 0..3 float4 groups, s = 0..3), so each operand fragment is one ds_read_b128 per 4 k-steps;
// rows padded to 36 floats: conflict-free for the ds_read_b128 lane groups.
//
// Persistent: a block walks the output tiles slot, slot + G, slot + 2G, ... (G = gridDim.x, two
// blocks per CU), and its K tiles form one flat pipeline across tile boundaries (the next tile's
// first K tile is fetched while this tile's last one is multiplied; the epilogue's stores drain
// while the next tile's MFMAs run).  Slots are XCD-aware: block b runs on XCD b % 8 and takes slot
// (b % 8) G/8 + b / 8, so the n/128 column tiles of a row band are computed at the same time on
// ONE XCD and share the A rows through its L2.  G is a multiple of n/128, so a block always owns
// the same column tile: its bias-gradient column sums stay in registers over all its tiles.  The
// epilogue goes through LDS so that global stores (and, backward, the y loads) are 16 B per lane.
namespace vgemm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// EPI_TANH_OUT: EPI_TANH for the last hidden layer (n = 256, a block holds whole rows) plus the
// output layer folded in (ppo…:104-111's last nn.Linear): the block also writes, per 64-column wave
// slice, the partial dot products of its tanh rows with the output layer's weight
// (out_part[slice][row][a], a < KO), so out = sum over the 4 slices + bias without reading y again.
enum { EPI_TANH = 0, EPI_DTANH = 1, EPI_TANH_OUT = 2 };

// tanh(z): odd Taylor polynomial to z^9 for |z| < 0.3 (truncation < 0.6 ulp there; the exponential
// form below would cancel in 1 - t), else sign(z) (1 - t) / (1 + t), t = 2^(-2|z| log2 e), on the
// hardware exp2 / rcp.  Within a few ulp of tanhf (tests/test_update.py).
__device__ __forceinline__ float tanh_f32(float z) {
  const float a = fabsf(z), s = z * z;
  const float poly = z + z * s * (-0.333333343f + s * (0.133333340f + s * (-0.0539682545f + s * 0.0218694885f)));
  const float t = __builtin_amdgcn_exp2f(-2.8853900817779268f * a);
  const float ex = copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), z);
  return a < 0.3f ? poly : ex;
}

constexpr int kKS = 32, kLS = kKS + 4;  // K tile, LDS row stride (floats; conflict-free ds_read_b128 groups)
constexpr int kES = 72;  // epilogue scratch row stride (floats)

// Block geometry: BM x BN output tile, WM x WN waves, each a (BM/WM) x (BN/WN) block of 32x32 MFMA tiles.
template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int THREADS = 64 * WM * WN;
  static constexpr int WROWS = BM / WM, WCOLS = BN / WN;
  static constexpr int TM = WROWS / 32, TN = WCOLS / 32;
  static constexpr int LDSF = 2 * (BM + BN) * kLS;  // two K-tile buffers
  static constexpr int SCR = WM * WN * 32 * kES;  // epilogue scratch, inside K-tile buffer 1
  static_assert(SCR <= (BM + BN) * kLS, "epilogue scratch must fit one K-tile buffer");
  static constexpr int LROWS = THREADS / 8;          // rows one staging pass covers (8 float4 per 32-float row)
  static constexpr int RA = BM / LROWS, RB = BN / LROWS;
  static constexpr int BLOCKS_PER_CU = LDSF * 4 * 2 <= 160 * 1024 ? 2 : 1;
  static_assert(WCOLS == 64, "the epilogue streams 64-column wave tiles");
  static_assert(RA * LROWS == BM && RB * LROWS == BN, "staging passes must tile the block");
};
using Cfg128 = Cfg<128, 128, 2, 2>;     // 4 waves, 72 KB LDS: two blocks per CU
using Cfg256 = Cfg<256, 256, 2, 4>;     // 8 waves of 128 x 64, 144 KB LDS: one block per CU
// (measured and not kept: 8-wave 256 x 128 / 128 x 256 blocks, profiles/r02_gemm_{fwd,bwd}_tiles*.log)

struct GemmArgs {
  int64_t rows;
  int32_t n, k;
  const float* a;     // (rows, k)
  const float* b;     // (n, k)
  const float* bias;  // EPI_TANH: (n)
  const float* y;     // EPI_DTANH: (rows, n), the tanh output the gradient passes through
  float* out;         // (rows, n)
  float* partial;     // EPI_DTANH: (G / (n / BN), n) column sums of out
  int64_t tiles;      // ceil(rows / BM) * (n / BN) output tiles, row band major
  const float* w_out; // EPI_TANH_OUT: the output layer's weight (KO, n)
  float* out_part;    // EPI_TANH_OUT: (n / 64, rows, KO) partial output-layer sums
};

// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r + 15): xor 1 and 2 by quad permutes, then the
// half-row and row mirrors (which act as xor 4 and xor 8 once every quad, then every half, is
// uniform); every lane of the row ends with the row's sum, added in one fixed order.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f32<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f32<0x141>(v);  // row_half_mirror
  v += dpp_f32<0x140>(v);  // row_mirror
  return v;
}

// One wave's (TM x 32) x 64 output block, 32 x 64 at a time through the wave's LDS scratch (32 x kES
// floats), so that every global access is a 16-B piece of a 256-B row segment.  C/D map of a 32x32
// MFMA tile: col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5).  Row stride kES = 72: the
// two row halves of a ds_write_b32 land 32 banks apart and each 16-lane ds_read_b128 group reads 64
// consecutive dwords (conflict-free both ways).  EPI_TANH: out = tanh(acc + bias); EPI_DTANH:
// out = acc * (1 - y^2) and csum += out (this lane's 4 columns).
template <int EPI, int TM, int TN, bool MASK = true, int KO = 0>
__device__ __forceinline__ void store_tile(const GemmArgs& p, f32x16 (&acc)[TM][TN], float* scr, int64_t rowb0, int colw,
                                           float4& csum, const float* wo_lds = nullptr) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int er = lane >> 4, ec = (lane & 15) * 4;  // reader: rows er + 4q, columns ec..ec+3
  const int64_t M = p.rows;
  static_assert(EPI != EPI_TANH_OUT || (KO > 0 && !MASK), "EPI_TANH_OUT: exact shapes, KO output columns");
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t rowb = rowb0 + i * 32;
    // EPI_DTANH: y of rows er + 4q, four rows in flight (loaded before the LDS round trip, then each
    // slot refilled with the row four steps ahead as it is consumed)
    auto yload = [&](int q) {
      const int64_t row = rowb + er + 4 * q;
      return (!MASK || row < M) ? *reinterpret_cast<const float4*>(p.y + row * p.n + colw + ec)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    float4 yv[4];
    if constexpr (EPI == EPI_DTANH) {
#pragma unroll
      for (int q = 0; q < 4; ++q) yv[q] = yload(q);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float bcol = EPI != EPI_DTANH ? p.bias[colw + j * 32 + r] : 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float v = acc[i][j][e];
        if constexpr (EPI != EPI_DTANH) v = tanh_f32(v + bcol);
        scr[((e & 3) + 8 * (e >> 2) + 4 * h) * kES + j * 32 + r] = v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float4 v = *reinterpret_cast<const float4*>(scr + (er + 4 * q) * kES + ec);
      const int64_t row = rowb + er + 4 * q;
      if constexpr (EPI == EPI_DTANH) {
        const float4 yq = yv[q & 3];
        if (q < 4) yv[q] = yload(q + 4);
        v = make_float4(v.x * fmaf(-yq.x, yq.x, 1.0f), v.y * fmaf(-yq.y, yq.y, 1.0f), v.z * fmaf(-yq.z, yq.z, 1.0f),
                        v.w * fmaf(-yq.w, yq.w, 1.0f));
        if (!MASK || row < M) vupd::add4(csum, v);
      }
      if (!MASK || row < M) {
        if constexpr (EPI == EPI_DTANH) {
          // the backward's gradient streams out nontemporally: 1-4 % faster on the three backward
          // shapes, no change on the forward (profiles/r02_gemm_epilogue_variants.log)
          __builtin_nontemporal_store((vupd::f32x4){v.x, v.y, v.z, v.w},
                                      reinterpret_cast<vupd::f32x4*>(p.out + row * p.n + colw + ec));
        } else {
          *reinterpret_cast<float4*>(p.out + row * p.n + colw + ec) = v;
        }
      }
      if constexpr (EPI == EPI_TANH_OUT) {
        // the output layer on this row's 64 columns of the slice: 4 products per lane, then the 16
        // lanes of the row; one lane writes the slice's partial sums (fixed order: deterministic)
#pragma unroll
        for (int a = 0; a < KO; ++a) {
          // the output weights of this lane's 4 columns, from the LDS copy (a global load here would
          // wait, by vmcnt's in-order count, for the K tiles prefetched behind it)
          const vupd::f32x4 wo = *reinterpret_cast<const vupd::f32x4*>(wo_lds + a * 256 + colw + ec);
          float d = v.x * wo[0];
          d = fmaf(v.y, wo[1], d);
          d = fmaf(v.z, wo[2], d);
          d = fmaf(v.w, wo[3], d);
          d = row16_sum(d);
          if ((lane & 15) == 0) p.out_part[((int64_t)(colw >> 6) * M + row) * KO + a] = d;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// EPI_DTANH: the block's column sums into partial row slot / nb — the 4 row groups of a wave (lanes
// ec/4, +16, +32, +48), then the WM row waves, in a fixed order (deterministic).  `red` is LDS the
// caller has released (a __syncthreads() before the call).
template <int WM, int BN>
__device__ __forceinline__ void write_colsums(const GemmArgs& p, float4 csum, float* red, int slot, int nb, int wm,
                                              int wcol) {
  const int tid = threadIdx.x, lane = tid & 63, er = lane >> 4, ec = (lane & 15) * 4;
  csum.x += __shfl_xor(csum.x, 16); csum.y += __shfl_xor(csum.y, 16);
  csum.z += __shfl_xor(csum.z, 16); csum.w += __shfl_xor(csum.w, 16);
  csum.x += __shfl_xor(csum.x, 32); csum.y += __shfl_xor(csum.y, 32);
  csum.z += __shfl_xor(csum.z, 32); csum.w += __shfl_xor(csum.w, 32);
  if (er == 0) *reinterpret_cast<float4*>(red + wm * BN + wcol + ec) = csum;
  __syncthreads();
  if (tid < BN) {
    float s = red[tid];
#pragma unroll
    for (int m = 1; m < WM; ++m) s += red[m * BN + tid];
    p.partial[(int64_t)(slot / nb) * p.n + (slot % nb) * BN + tid] = s;
  }
}

template <int EPI, class C, bool EXACT>
__global__ __launch_bounds__(C::THREADS, C::BLOCKS_PER_CU) void gemm_kernel(GemmArgs p) {
  constexpr int BM = C::BM, BN = C::BN, TM = C::TM, TN = C::TN, LROWS = C::LROWS;
  __shared__ float lds[C::LDSF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv / C::WN, wn = wv % C::WN;
  const int nb = p.n / BN;
  const int K = p.k, ktiles = (K + kKS - 1) / kKS;
  const int64_t M = p.rows;
  const int G = gridDim.x, tiles = (int)p.tiles;
  const int slot = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (slot >= tiles) return;  // whole block (the host sizes G <= tiles)
  int tile = slot;

  // loader: thread tid stages rows lr + LROWS i and floats lc..lc+3 of each K tile
  const int lr = tid >> 3, lc = (tid & 7) * 4;
  const int64_t KL = (int64_t)LROWS * K;
  const float* pa;  // this thread's first A row of the tile being fetched, at column lc
  const float* pb;
  int arows;        // rows of that tile below M
  auto set_fetch_tile = [&](int t) {
    const int64_t row0 = (int64_t)(t / nb) * BM;
    const int col0 = (t % nb) * BN;
    pa = p.a + (row0 + lr) * K + lc;
    pb = p.b + (int64_t)(col0 + lr) * K + lc;
    arows = (int)((M - row0) < BM ? (M - row0) : BM);
  };
  // EXACT (rows % BM == 0 and K % 32 == 0, the update's shapes but the first layer): plain loads whose
  // registers are first read by the LDS write at the end of the K tile, so they stay in flight
  // during the MFMAs.  Otherwise the masked form below, after which the compiler waits for the
  // loads before the MFMAs (measured: the global loads then cost ~11 %, a barrier-free probe ~7 %).
  auto gload = [&](float4 (&ra)[C::RA], float4 (&rb)[C::RB], int kt) {
    const int ko = kt * kKS;
    if constexpr (EXACT) {
      // loaded as a vector value (a float4 struct copy became a memcpy into a private array that
      // was not promoted to registers)
#pragma unroll
      for (int i = 0; i < C::RA; ++i) {
        const vupd::f32x4 v = *reinterpret_cast<const vupd::f32x4*>(pa + i * KL + ko);
        ra[i] = make_float4(v.x, v.y, v.z, v.w);
      }
#pragma unroll
      for (int i = 0; i < C::RB; ++i) {
        const vupd::f32x4 v = *reinterpret_cast<const vupd::f32x4*>(pb + i * KL + ko);
        rb[i] = make_float4(v.x, v.y, v.z, v.w);
      }
    } else {
      const bool kin = kt * kKS + lc < K;
#pragma unroll
      for (int i = 0; i < C::RA; ++i)
        ra[i] = (kin && lr + LROWS * i < arows) ? *reinterpret_cast<const float4*>(pa + i * KL + ko) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < C::RB; ++i)
        rb[i] = kin ? *reinterpret_cast<const float4*>(pb + i * KL + ko) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto swrite = [&](const float4 (&ra)[C::RA], const float4 (&rb)[C::RB], int buf) {
    float* As = lds + buf * (BM + BN) * kLS;
    float* Bs = As + BM * kLS;
#pragma unroll
    for (int i = 0; i < C::RA; ++i) *reinterpret_cast<float4*>(As + (lr + LROWS * i) * kLS + lc) = ra[i];
#pragma unroll
    for (int i = 0; i < C::RB; ++i) *reinterpret_cast<float4*>(Bs + (lr + LROWS * i) * kLS + lc) = rb[i];
  };

  f32x16 acc[TM][TN];
  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);  // EPI_DTANH: this lane's 4 column sums over all its tiles
  set_fetch_tile(tile);
  {
    float4 ra[C::RA], rb[C::RB];
    gload(ra, rb, 0);
    swrite(ra, rb, 0);
  }
  __syncthreads();
  const int r = lane & 31, h = lane >> 5;
  int buf = 0;
  for (;;) {
    const int next = tile + G;
    const bool has_next = next < tiles;
    const int64_t row0 = (int64_t)(tile / nb) * BM;
    const int col0 = (tile % nb) * BN;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = (f32x16){0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < ktiles; ++kt) {
      float4 ra[C::RA], rb[C::RB];  // the next K tile's operands, staged through registers
      // the next K tile of the flat pipeline: this tile's kt + 1, else the next tile's first
      const bool last = kt + 1 == ktiles;
      const bool more = !last || has_next;
      // one load site, no branch around it: the loaded registers then need no copies at a control
      // flow join (copies made the compiler wait for the loads before the MFMAs).  After the
      // block's last tile this re-fetches its first K tile, which is never written to LDS.
      if (last && has_next) set_fetch_tile(next);
      gload(ra, rb, last ? 0 : kt + 1);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs (the scheduler sinks them)
      const float* As = lds + buf * (BM + BN) * kLS + (wm * C::WROWS + r) * kLS + h * 16;
      const float* Bs = lds + buf * (BM + BN) * kLS + BM * kLS + (wn * C::WCOLS + r) * kLS + h * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 a4[TM], b4[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a4[i] = *reinterpret_cast<const float4*>(As + i * 32 * kLS + q * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) b4[j] = *reinterpret_cast<const float4*>(Bs + j * 32 * kLS + q * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const float av = s == 0 ? a4[i].x : s == 1 ? a4[i].y : s == 2 ? a4[i].z : a4[i].w;
              const float bv = s == 0 ? b4[j].x : s == 1 ? b4[j].y : s == 2 ? b4[j].z : b4[j].w;
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
            }
      }
      if (more) {
        swrite(ra, rb, buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }

    // epilogue through the free LDS buffer (buf ^ 1: every wave has passed the barrier after its last read)
    store_tile<EPI, TM, TN>(p, acc, lds + (buf ^ 1) * (BM + BN) * kLS + wv * (32 * kES), row0 + wm * C::WROWS,
                            col0 + wn * C::WCOLS, csum);
    if (!has_next) break;
    __syncthreads();  // the next tile's first swrite reuses the scratch buffer
    tile = next;
  }

  if constexpr (EPI == EPI_DTANH) {
    __syncthreads();  // every wave is done with the LDS buffers
    write_colsums<C::WM, BN>(p, csum, lds, slot, nb, wm, wn * C::WCOLS);
  }
}

// Exact shapes (rows % BM == 0, K % 64 == 0), loads TWO K tiles ahead: two
// register sets alternate with the two LDS buffers, so a K tile's global loads are issued two MFMA
// phases before the LDS write that consumes them (one phase in gemm_kernel: the HBM-missing A rows
// of a new row band then stall that write, and through the barrier every wave of the block).  K
// tile g of the block's flat sequence (its tiles' K tiles back to back): MFMAs on LDS[g & 1];
// write R[(g + 1) & 1] (= K tile g + 1) into LDS[(g + 1) & 1]; barrier; load K tile g + 3 into
// R[(g + 1) & 1].  The fetch cursor advances its pointers by one K tile (32 floats) per load and
// recomputes them only at a tile change.
template <int EPI, class C, int KO = 0>
__global__ __launch_bounds__(C::THREADS, C::BLOCKS_PER_CU) void gemm_kernel_d2(GemmArgs p) {
  constexpr int BM = C::BM, BN = C::BN, TM = C::TM, TN = C::TN, LROWS = C::LROWS, RA = C::RA, RB = C::RB;
  static_assert(EPI != EPI_TANH_OUT || BN == 256, "EPI_TANH_OUT: blocks of whole 256-wide rows");
  __shared__ float lds[C::LDSF];
  __shared__ float wo_lds[KO > 0 ? KO * 256 : 1];  // EPI_TANH_OUT: the output layer's weight (KO, 256)
  if constexpr (KO > 0)
    for (int i = threadIdx.x; i < KO * 256; i += C::THREADS) wo_lds[i] = p.w_out[i];  // published by the first barrier
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv / C::WN, wn = wv % C::WN;
  const int nb = p.n / BN;
  const int K = p.k, ktiles = K / kKS;  // even (K % 64 == 0)
  const int G = gridDim.x, tiles = (int)p.tiles;
  const int slot = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (slot >= tiles) return;

  const int lr = tid >> 3, lc = (tid & 7) * 4;
  const int64_t KL = (int64_t)LROWS * K;
  // fetch cursor: the next K tile to load (tile f_tile, k tile f_kt); past the last tile it keeps
  // re-loading the last one (in bounds, never multiplied)
  int f_tile = slot, f_kt = 0;
  const float* fa;
  const float* fb;
  auto point = [&](int t) {
    fa = p.a + ((int64_t)(t / nb) * BM + lr) * K + lc;
    fb = p.b + ((int64_t)((t % nb) * BN) + lr) * K + lc;
  };
  point(f_tile);
  auto advance = [&]() {
    if (++f_kt < ktiles) {
      fa += kKS;
      fb += kKS;
    } else if (f_tile + G < tiles) {
      f_kt = 0;
      f_tile += G;
      point(f_tile);
    } else {
      f_kt = ktiles - 1;  // stay on the block's last K tile
    }
  };
  auto gload = [&](float4 (&ra)[RA], float4 (&rb)[RB]) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const vupd::f32x4 v = *reinterpret_cast<const vupd::f32x4*>(fa + i * KL);
      ra[i] = make_float4(v.x, v.y, v.z, v.w);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const vupd::f32x4 v = *reinterpret_cast<const vupd::f32x4*>(fb + i * KL);
      rb[i] = make_float4(v.x, v.y, v.z, v.w);
    }
    advance();
  };
  auto swrite = [&](const float4 (&ra)[RA], const float4 (&rb)[RB], int buf) {
    float* As = lds + buf * (BM + BN) * kLS;
    float* Bs = As + BM * kLS;
#pragma unroll
    for (int i = 0; i < RA; ++i) *reinterpret_cast<float4*>(As + (lr + LROWS * i) * kLS + lc) = ra[i];
#pragma unroll
    for (int i = 0; i < RB; ++i) *reinterpret_cast<float4*>(Bs + (lr + LROWS * i) * kLS + lc) = rb[i];
  };
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[TM][TN];
  auto mfma_tile = [&](int buf) {
    const float* As = lds + buf * (BM + BN) * kLS + (wm * C::WROWS + r) * kLS + h * 16;
    const float* Bs = lds + buf * (BM + BN) * kLS + BM * kLS + (wn * C::WCOLS + r) * kLS + h * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 a4[TM], b4[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a4[i] = *reinterpret_cast<const float4*>(As + i * 32 * kLS + q * 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) b4[j] = *reinterpret_cast<const float4*>(Bs + j * 32 * kLS + q * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const float av = s == 0 ? a4[i].x : s == 1 ? a4[i].y : s == 2 ? a4[i].z : a4[i].w;
            const float bv = s == 0 ? b4[j].x : s == 1 ? b4[j].y : s == 2 ? b4[j].z : b4[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
    }
  };

  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ra0[RA], rb0[RB], ra1[RA], rb1[RB];
  gload(ra0, rb0);  // K tile 0
  swrite(ra0, rb0, 0);
  gload(ra1, rb1);  // K tile 1
  gload(ra0, rb0);  // K tile 2
  __syncthreads();
  int tile = slot;
  for (;;) {
    const int next = tile + G;
    const bool has_next = next < tiles;
    const int64_t row0 = (int64_t)(tile / nb) * BM;
    const int col0 = (tile % nb) * BN;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = (f32x16){0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // K tiles in pairs: even g (LDS 0, writes R1 -> LDS 1, reloads R1), odd g (LDS 1, R0 -> LDS 0)
    for (int kt = 0; kt < ktiles; kt += 2) {
      mfma_tile(0);
      swrite(ra1, rb1, 1);
      __syncthreads();
      gload(ra1, rb1);
      mfma_tile(1);
      swrite(ra0, rb0, 0);
      __syncthreads();
      gload(ra0, rb0);
    }
    // epilogue through LDS buffer 1: every wave has passed the barrier after its last read of it,
    // and the next tile's first K tile sits in LDS 0
    // backward, exact shapes: no row masks (their branches made the compiler drain vmcnt to 0, i.e.
    // wait for the K tiles prefetched two ahead, at every y load; the forward measured ~1 % slower
    // without them, profiles/r02_gemm_epilogue_variants.log)
    store_tile<EPI, TM, TN, EPI == EPI_TANH, KO>(p, acc, lds + (BM + BN) * kLS + wv * (32 * kES),
                                                 row0 + wm * C::WROWS, col0 + wn * C::WCOLS, csum, wo_lds);
    if (!has_next) break;
    __syncthreads();  // the next tile's second K tile is written into LDS 1 (the scratch)
    tile = next;
  }
  if constexpr (EPI == EPI_DTANH) {
    __syncthreads();
    write_colsums<C::WM, BN>(p, csum, lds, slot, nb, wm, wn * C::WCOLS);
  }
}

// The persistent grid is sized for MI355X (256 CUs) on every device: a block walks its tiles however
// many blocks are resident, so the grid -- and with it the bias-gradient partial layout and its
// summation order -- does not depend on the device the call runs on.
constexpr int kGridCus = 256;


// the launch plan of one GEMM: kernel, output tiles, grid
struct Plan {
  int kind;  // 0 Cfg128, 1 Cfg256
  int bn;
  int64_t tiles, grid;
};

// Exact shapes: rows % 128 == 0 and K % 32 == 0 (the update's layers but the first).
static bool exact_shape(int64_t rows, int32_t k, int bm) { return rows % bm == 0 && k % kKS == 0; }

static Plan plan(int64_t rows, int32_t k, int32_t n, bool forward) {
  Plan pl;
  // Exact shapes run the 128 x 128 blocks with unmasked, pipelined loads (fastest there); the masked
  // form is fastest on 256 x 256 blocks (profiles/r01_gemm_fused_bench.log).
  const bool exact = exact_shape(rows, k, Cfg128::BM);
  pl.kind = (!exact && n % 256 == 0) ? 1 : 0;
  // the forward's exact shapes on 256 x 256 blocks with the two-deep pipeline: 123-134 TF vs 116-127 on
  // 128 x 128 (profiles/r02_gemm_d2c256.log); the backward's epilogue needs more registers than a
  // 256 x 256 block leaves (it spills), so it stays on 128 x 128
  if (forward && exact && rows % Cfg256::BM == 0 && k % (2 * kKS) == 0 && n % 256 == 0) pl.kind = 1;
  const int bm = pl.kind == 1 ? Cfg256::BM : Cfg128::BM;
  const int bpc = pl.kind == 1 ? Cfg256::BLOCKS_PER_CU : Cfg128::BLOCKS_PER_CU;
  pl.bn = pl.kind == 1 ? Cfg256::BN : Cfg128::BN;
  const int nb = n / pl.bn;
  pl.tiles = (rows + bm - 1) / bm * nb;
  // persistent: min(tiles, blocks_per_cu x CUs), the latter rounded down to a multiple of 8 (XCD
  // slots) and of nb (a fixed column tile per block)
  int64_t g = (int64_t)kGridCus * bpc;
  g -= g % (8 * (int64_t)nb);
  pl.grid = (g > 0 && g < pl.tiles) ? g : pl.tiles;
  return pl;
}

static bool shape_ok(int64_t rows, int32_t k, int32_t n) {
  return rows >= 0 && rows <= (int64_t(1) << 40) && k >= 4 && k % 4 == 0 && k <= 65536 && n >= 128 && n % 128 == 0 &&
         n <= 65536 && (rows + 127) / 128 * (n / 128) <= 0x7fff0000;  // tile + grid stays in int
}


template <int EPI, bool EXACT>
static void launch_kind(const GemmArgs& a, const Plan& pl, hipStream_t s) {
  const dim3 grid((unsigned)pl.grid);
  if (EXACT && pl.kind == 0 && a.k % (2 * kKS) == 0) {
    hipLaunchKernelGGL((gemm_kernel_d2<EPI, Cfg128>), grid, dim3(Cfg128::THREADS), 0, s, a);
    return;
  }
  if (EPI == EPI_TANH && EXACT && pl.kind == 1 && a.k % (2 * kKS) == 0) {
    hipLaunchKernelGGL((gemm_kernel_d2<EPI_TANH, Cfg256>), grid, dim3(Cfg256::THREADS), 0, s, a);
    return;
  }
  if (pl.kind == 1)
    hipLaunchKernelGGL((gemm_kernel<EPI, Cfg256, EXACT>), grid, dim3(Cfg256::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<EPI, Cfg128, EXACT>), grid, dim3(Cfg128::THREADS), 0, s, a);
}

template <int EPI>
static int launch(void* stream, const GemmArgs& a0, const Plan& pl) {
  GemmArgs a = a0;
  a.tiles = pl.tiles;
  if (exact_shape(a.rows, a.k, pl.kind == 1 ? Cfg256::BM : Cfg128::BM))
    launch_kind<EPI, true>(a, pl, (hipStream_t)stream);
  else
    launch_kind<EPI, false>(a, pl, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

// ---- the first hidden layer's forward: y = tanh(x W^T + b), K = 52 (<= 64), N = 256 --------------
// At 2,097,152 rows this is 0.44 GB in, 2.1 GB out and 56 GFLOP: the K loop is two K tiles and the
// epilogue writes 8x what the loop reads, and the tiled GEMM ran them back to back (0.93-1.15 ms).
// Here W^T (K x 256, <= 64 KB) is staged into LDS once per block and every wave works alone on
// 32-row slabs: its x values straight from global memory (one float4 per lane and 8-wide K step),
// 8 column tiles x 4 K steps of v_mfma_f32_32x32x2_f32 per float4, then bias + tanh and the stores;
// with no barrier after the staging, one wave's tanh and stores run beside the other waves' MFMAs.
// MFMA step (j, s): lane half h contributes k = 8j + 4h + s.
constexpr int kFlThreads = 256;

static bool first_layer_ok(int32_t k, int32_t n) { return n == 256 && k % 4 == 0 && k > 48 && k <= 64; }

template <int J>
__global__ __launch_bounds__(kFlThreads, 2) void first_layer_kernel(int64_t rows, int k, const float* __restrict__ x,
                                                                    const float* __restrict__ w,
                                                                    const float* __restrict__ bias,
                                                                    float* __restrict__ y) {
  // wl[((kk * 2 + c) * 32 + r) * 4 + q] = w[32 (4c + q) + r][kk] (zero for kk >= k): a lane's 8 column
  // tiles of one K row are two consecutive float4s, consecutive lanes 16 B apart
  __shared__ float4 wl[8 * J * 2 * 32];
  for (int i = threadIdx.x; i < 8 * J * 256; i += kFlThreads) {
    const int q = i & 3, rr = (i >> 2) & 31, c = (i >> 7) & 1, kk = i >> 8;
    reinterpret_cast<float*>(wl)[i] = kk < k ? w[(int64_t)(32 * (4 * c + q) + rr) * k + kk] : 0.0f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  float bcol[8];
#pragma unroll
  for (int ct = 0; ct < 8; ++ct) bcol[ct] = bias[ct * 32 + r];
  const int64_t slabs = (rows + 31) / 32, step = (int64_t)gridDim.x * (kFlThreads / 64);
  auto load_x = [&](int64_t sl, float4 (&xv)[J]) __attribute__((always_inline)) {
    const int64_t row = sl * 32 + r;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int kk = 8 * j + 4 * h;
      xv[j] = (row < rows && kk < k) ? *reinterpret_cast<const float4*>(x + row * k + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // (Measured and not kept, profiles/r02_gemm_first_layer*.log: a software pipeline running one half
  // slab's MFMAs beside the other half's epilogue -- both accumulator sets, so one wave per SIMD:
  // 899 vs 804 us; the second block of each CU started half a slab late: no change.)
  int64_t sl = (int64_t)blockIdx.x * (kFlThreads / 64) + wv;
  float4 xv[J];
  if (sl < slabs) load_x(sl, xv);
  for (; sl < slabs; sl += step) {
    float4 xc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) xc[j] = xv[j];
    if (sl + step < slabs) load_x(sl + step, xv);  // the next slab's x lands during this slab
    f32x16 acc[8];
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
      acc[ct] = (f32x16){0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const float av = s4 == 0 ? xc[j].x : s4 == 1 ? xc[j].y : s4 == 2 ? xc[j].z : xc[j].w;
        const float4* wr = wl + ((8 * j + 4 * h + s4) * 2) * 32 + r;
        const float4 b0 = wr[0], b1 = wr[32];
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[ct], acc[ct], 0, 0, 0);
      }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t orow = sl * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (orow < rows) {
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) y[orow * 256 + ct * 32 + r] = tanh_f32(acc[ct][e] + bcol[ct]);
      }
    }
  }
}

// ---- the output layer's backward: k_next = 4 or 8 (the 1, 2 or 6 output columns, zero-padded) ------
// gz = (gz_next W_next) * (1 - y^2) with a contraction of 4 or 8 is a streaming pass over y and gz
// (2 x 4 B per element, ~2 k FLOP per element), not a GEMM: on the masked MFMA path it padded K to
// a 32-wide K tile and ran the MFMAs, then the epilogue, one after the other (1.02 ms at 2,097,152 x
// 256, 4.1 TB/s).  Here every thread owns 4 columns with their k_next weights in registers, a block
// walks a contiguous band of rows with four rows in flight per thread, gz streams out
// nontemporally, and the block's column sums land in partial[block] (one fixed summation order).
constexpr int kSmallThreads = 256;
constexpr int kSmallMaxBlocks = 2048;

struct SmallPlan {
  int64_t rows_per_block, blocks;
};

static bool small_k(int32_t k_next, int32_t n) {
  return (k_next == 4 || k_next == 8) && 1024 % n == 0;
}

static SmallPlan small_plan(int64_t rows, int32_t n) {
  const int64_t rpp = kSmallThreads / (n / 4);  // rows one pass of the block covers
  int64_t g = (rows + rpp - 1) / rpp;
  if (g > kSmallMaxBlocks) g = kSmallMaxBlocks;
  int64_t per = (rows + g - 1) / g;
  per = (per + rpp - 1) / rpp * rpp;
  return SmallPlan{per, (rows + per - 1) / per};
}

// WG (vss_output_backward): the same pass also accumulates the output layer's weight gradient
// g_out^T y (its input is y) from the values it already holds, as per-block partials (KN x n).
template <int KN, bool WG = false>
__global__ __launch_bounds__(kSmallThreads) void dtanh_small_k_kernel(int64_t rows, int n, const float* __restrict__ g,
                                                                      const float* __restrict__ wt,
                                                                      const float* __restrict__ y, float* __restrict__ out,
                                                                      float* __restrict__ partial, int64_t per,
                                                                      float* __restrict__ wpartial = nullptr) {
  __shared__ float4 red[kSmallThreads];
  float4 wacc[WG ? KN : 1];
#pragma unroll
  for (int a = 0; a < (WG ? KN : 1); ++a) wacc[a] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int tpr = n >> 2, rpp = kSmallThreads / tpr;
  const int tid = threadIdx.x, c = (tid % tpr) * 4, ro = tid / tpr;
  float w[4][KN];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int a = 0; a < KN; ++a) w[j][a] = wt[(int64_t)(c + j) * KN + a];
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  constexpr int U = 4;
  for (int64_t rb = r0 + ro; rb < r1; rb += (int64_t)U * rpp) {
    float4 yv[U], gv[U][KN / 4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = rb + (int64_t)u * rpp;
      if (row < r1) {
        yv[u] = *reinterpret_cast<const float4*>(y + row * n + c);
#pragma unroll
        for (int q = 0; q < KN / 4; ++q) gv[u][q] = *reinterpret_cast<const float4*>(g + row * KN + 4 * q);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = rb + (int64_t)u * rpp;
      if (row < r1) {
        const float* gr = reinterpret_cast<const float*>(gv[u]);
        float acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = gr[0] * w[j][0];
#pragma unroll
          for (int a = 1; a < KN; ++a) t = fmaf(gr[a], w[j][a], t);
          acc[j] = t;
        }
        const float4 yq = yv[u];
        const vupd::f32x4 v = {acc[0] * fmaf(-yq.x, yq.x, 1.0f), acc[1] * fmaf(-yq.y, yq.y, 1.0f),
                               acc[2] * fmaf(-yq.z, yq.z, 1.0f), acc[3] * fmaf(-yq.w, yq.w, 1.0f)};
        __builtin_nontemporal_store(v, reinterpret_cast<vupd::f32x4*>(out + row * n + c));
        cs.x += v[0]; cs.y += v[1]; cs.z += v[2]; cs.w += v[3];
        if constexpr (WG) {
#pragma unroll
          for (int a = 0; a < KN; ++a) {
            wacc[a].x = fmaf(gr[a], yq.x, wacc[a].x); wacc[a].y = fmaf(gr[a], yq.y, wacc[a].y);
            wacc[a].z = fmaf(gr[a], yq.z, wacc[a].z); wacc[a].w = fmaf(gr[a], yq.w, wacc[a].w);
          }
        }
      }
    }
  }
  red[tid] = cs;
  __syncthreads();
  if (tid < tpr) {
    float4 s4 = red[tid];
    for (int m = 1; m < rpp; ++m) vupd::add4(s4, red[m * tpr + tid]);
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.x * n + c) = s4;
  }
  if constexpr (WG) {
#pragma unroll
    for (int a = 0; a < KN; ++a) {
      __syncthreads();
      red[tid] = wacc[a];
      __syncthreads();
      if (tid < tpr) {
        float4 s4 = red[tid];
        for (int m = 1; m < rpp; ++m) vupd::add4(s4, red[m * tpr + tid]);
        *reinterpret_cast<float4*>(wpartial + ((int64_t)blockIdx.x * KN + a) * n + c) = s4;
      }
    }
  }
}

// The direct form (vss_output_backward_direct, the update's minibatch without autograd): g_out read as
// the loss wrote it (rows, KO), w_out as nn.Linear holds it (KO, n) -- no padded copies -- and blocks of
// 16 waves, at most kDirMaxBlocks of them, so that the partials (one row of column sums and KO rows of
// the weight gradient per block) are few enough for the backward's one vss_sum_parts launch.
constexpr int kDirThreads = 1024;
constexpr int kDirMaxBlocks = 256;

static SmallPlan direct_plan(int64_t rows, int32_t n) {
  const int64_t rpp = kDirThreads / (n / 4);
  int64_t g = (rows + rpp - 1) / rpp;
  if (g > kDirMaxBlocks) g = kDirMaxBlocks;
  int64_t per = (rows + g - 1) / g;
  per = (per + rpp - 1) / rpp * rpp;
  return SmallPlan{per, (rows + per - 1) / per};
}

template <int KO>
__global__ __launch_bounds__(kDirThreads) void output_backward_direct_kernel(int64_t rows, int n,
                                                                             const float* __restrict__ g,
                                                                             const float* __restrict__ w,
                                                                             const float* __restrict__ y,
                                                                             float* __restrict__ out,
                                                                             float* __restrict__ partial, int64_t per,
                                                                             float* __restrict__ wpartial) {
  __shared__ float4 red[kDirThreads];
  float4 wacc[KO];
#pragma unroll
  for (int a = 0; a < KO; ++a) wacc[a] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int tpr = n >> 2, rpp = kDirThreads / tpr;
  const int tid = threadIdx.x, c = (tid % tpr) * 4, ro = tid / tpr;
  float wr[4][KO];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int a = 0; a < KO; ++a) wr[j][a] = w[(int64_t)a * n + c + j];
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  constexpr int U = KO == 1 ? 8 : (KO == 2 ? 6 : (KO <= 4 ? 4 : 2));  // rows in flight per thread (no spill at 1,024 threads)
  for (int64_t rb = r0 + ro; rb < r1; rb += (int64_t)U * rpp) {
    float4 yv[U];
    float gv[U][KO];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = rb + (int64_t)u * rpp;
      if (row < r1) {
        yv[u] = *reinterpret_cast<const float4*>(y + row * n + c);
#pragma unroll
        for (int a = 0; a < KO; ++a) gv[u][a] = g[row * KO + a];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = rb + (int64_t)u * rpp;
      if (row < r1) {
        float acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = gv[u][0] * wr[j][0];
#pragma unroll
          for (int a = 1; a < KO; ++a) t = fmaf(gv[u][a], wr[j][a], t);
          acc[j] = t;
        }
        const float4 yq = yv[u];
        const vupd::f32x4 v = {acc[0] * fmaf(-yq.x, yq.x, 1.0f), acc[1] * fmaf(-yq.y, yq.y, 1.0f),
                               acc[2] * fmaf(-yq.z, yq.z, 1.0f), acc[3] * fmaf(-yq.w, yq.w, 1.0f)};
        __builtin_nontemporal_store(v, reinterpret_cast<vupd::f32x4*>(out + row * n + c));
        cs.x += v[0]; cs.y += v[1]; cs.z += v[2]; cs.w += v[3];
#pragma unroll
        for (int a = 0; a < KO; ++a) {
          wacc[a].x = fmaf(gv[u][a], yq.x, wacc[a].x); wacc[a].y = fmaf(gv[u][a], yq.y, wacc[a].y);
          wacc[a].z = fmaf(gv[u][a], yq.z, wacc[a].z); wacc[a].w = fmaf(gv[u][a], yq.w, wacc[a].w);
        }
      }
    }
  }
  red[tid] = cs;
  __syncthreads();
  if (tid < tpr) {
    float4 s4 = red[tid];
    for (int m = 1; m < rpp; ++m) vupd::add4(s4, red[m * tpr + tid]);
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.x * n + c) = s4;
  }
#pragma unroll
  for (int a = 0; a < KO; ++a) {
    __syncthreads();
    red[tid] = wacc[a];
    __syncthreads();
    if (tid < tpr) {
      float4 s4 = red[tid];
      for (int m = 1; m < rpp; ++m) vupd::add4(s4, red[m * tpr + tid]);
      *reinterpret_cast<float4*>(wpartial + ((int64_t)blockIdx.x * KO + a) * n + c) = s4;
    }
  }
}

}  // namespace vgemm

extern "C" {

static bool tanh_grad_cols_ok(int32_t cols) {
  return cols == 64 || cols == 128 || cols == 256 || cols == 512 || cols == 1024;
}

static bool misaligned(const void* p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) != 0; }

int64_t vss_tanh_grad_chunks(int64_t rows, int32_t cols) {
  return (rows < 0 || !tanh_grad_cols_ok(cols)) ? -1 : vupd::n_blocks(rows, cols);
}

int vss_tanh_grad_bias(void* stream, int64_t rows, int32_t cols, const float* grad_out, const float* y,
                       float* grad_in, float* bias_partial) {
  if (rows < 0 || rows > (int64_t(1) << 40) || misaligned(grad_out) || misaligned(y) || misaligned(grad_in) ||
      misaligned(bias_partial))
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

int vss_linear_tanh(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                    const float* bias, float* y) {
  if (!vgemm::shape_ok(rows, k_in, n_out) || misaligned(x) || misaligned(w) || misaligned(y) || !bias)
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  if (vgemm::first_layer_ok(k_in, n_out)) {
    const int64_t slabs = (rows + 31) / 32, per_block = vgemm::kFlThreads / 64;
    int64_t g = (slabs + per_block - 1) / per_block;
    if (g > 2 * vgemm::kGridCus) g = 2 * vgemm::kGridCus;  // two blocks (two waves per SIMD) per CU
    if (k_in > 56)
      hipLaunchKernelGGL(vgemm::first_layer_kernel<8>, dim3((unsigned)g), dim3(vgemm::kFlThreads), 0, (hipStream_t)stream,
                         rows, k_in, x, w, bias, y);
    else
      hipLaunchKernelGGL(vgemm::first_layer_kernel<7>, dim3((unsigned)g), dim3(vgemm::kFlThreads), 0, (hipStream_t)stream,
                         rows, k_in, x, w, bias, y);
    return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
  }
  const vgemm::GemmArgs a{rows, n_out, k_in, x, w, bias, nullptr, y, nullptr, 0, nullptr, nullptr};
  return vgemm::launch<vgemm::EPI_TANH>(stream, a, vgemm::plan(rows, k_in, n_out, true));
}

int vss_linear_tanh_out(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                        const float* bias, float* y, int32_t k_out, const float* w_out, float* out_part) {
  if (!vgemm::shape_ok(rows, k_in, n_out) || misaligned(x) || misaligned(w) || misaligned(y) || !bias ||
      misaligned(w_out) || !out_part)
    return VSS_E_ARG;
  // the forward's 256 x 256 blocks (whole 256-wide rows per block), exact shapes only
  if (n_out != 256 || rows % 256 != 0 || k_in % 64 != 0 || !(k_out == 1 || k_out == 2 || k_out == 6)) return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const vgemm::Plan pl = vgemm::plan(rows, k_in, n_out, true);
  if (pl.kind != 1) return VSS_E_ARG;
  vgemm::GemmArgs a{rows, n_out, k_in, x, w, bias, nullptr, y, nullptr, pl.tiles, w_out, out_part};
  const dim3 grid((unsigned)pl.grid), block(vgemm::Cfg256::THREADS);
  hipStream_t s = (hipStream_t)stream;
  if (k_out == 1) hipLaunchKernelGGL((vgemm::gemm_kernel_d2<vgemm::EPI_TANH_OUT, vgemm::Cfg256, 1>), grid, block, 0, s, a);
  else if (k_out == 2) hipLaunchKernelGGL((vgemm::gemm_kernel_d2<vgemm::EPI_TANH_OUT, vgemm::Cfg256, 2>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((vgemm::gemm_kernel_d2<vgemm::EPI_TANH_OUT, vgemm::Cfg256, 6>), grid, block, 0, s, a);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int64_t vss_linear_tanh_backward_chunks(int64_t rows, int32_t k_next, int32_t n_out) {
  if (!vgemm::shape_ok(rows, k_next, n_out)) return -1;
  if (rows == 0) return 0;
  if (vgemm::small_k(k_next, n_out)) return vgemm::small_plan(rows, n_out).blocks;
  const vgemm::Plan pl = vgemm::plan(rows, k_next, n_out, false);
  return pl.grid / (n_out / pl.bn);
}

int vss_linear_tanh_backward(void* stream, int64_t rows, int32_t k_next, int32_t n_out, const float* grad_next,
                             const float* w_next_t, const float* y, float* grad_in, float* bias_partial) {
  if (!vgemm::shape_ok(rows, k_next, n_out) || misaligned(grad_next) || misaligned(w_next_t) || misaligned(y) ||
      misaligned(grad_in) || misaligned(bias_partial))
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  if (vgemm::small_k(k_next, n_out)) {
    const vgemm::SmallPlan sp = vgemm::small_plan(rows, n_out);
    const dim3 grid((unsigned)sp.blocks), block(vgemm::kSmallThreads);
    if (k_next == 4)
      hipLaunchKernelGGL(vgemm::dtanh_small_k_kernel<4>, grid, block, 0, (hipStream_t)stream, rows, n_out, grad_next,
                         w_next_t, y, grad_in, bias_partial, sp.rows_per_block);
    else
      hipLaunchKernelGGL(vgemm::dtanh_small_k_kernel<8>, grid, block, 0, (hipStream_t)stream, rows, n_out, grad_next,
                         w_next_t, y, grad_in, bias_partial, sp.rows_per_block);
    return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
  }
  const vgemm::GemmArgs a{rows, n_out, k_next, grad_next, w_next_t, nullptr, y, grad_in, bias_partial, 0, nullptr, nullptr};
  return vgemm::launch<vgemm::EPI_DTANH>(stream, a, vgemm::plan(rows, k_next, n_out, false));
}

int64_t vss_output_backward_chunks(int64_t rows, int32_t k_pad, int32_t n) {
  if (rows < 0 || rows > (int64_t(1) << 40) || (k_pad != 4 && k_pad != 8) || n < 128 || n % 128 != 0 || 1024 % n != 0)
    return -1;
  return rows == 0 ? 0 : vgemm::small_plan(rows, n).blocks;
}

int vss_output_backward(void* stream, int64_t rows, int32_t k_pad, int32_t n, const float* g_out, const float* w_out_t,
                        const float* y, float* grad_in, float* bias_partial, float* wgrad_partial) {
  if (vss_output_backward_chunks(rows, k_pad, n) < 0 || misaligned(g_out) || misaligned(w_out_t) || misaligned(y) ||
      misaligned(grad_in) || misaligned(bias_partial) || misaligned(wgrad_partial))
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const vgemm::SmallPlan sp = vgemm::small_plan(rows, n);
  const dim3 grid((unsigned)sp.blocks), block(vgemm::kSmallThreads);
  if (k_pad == 4)
    hipLaunchKernelGGL((vgemm::dtanh_small_k_kernel<4, true>), grid, block, 0, (hipStream_t)stream, rows, n, g_out,
                       w_out_t, y, grad_in, bias_partial, sp.rows_per_block, wgrad_partial);
  else
    hipLaunchKernelGGL((vgemm::dtanh_small_k_kernel<8, true>), grid, block, 0, (hipStream_t)stream, rows, n, g_out,
                       w_out_t, y, grad_in, bias_partial, sp.rows_per_block, wgrad_partial);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

static bool output_direct_ok(int64_t rows, int32_t k_out, int32_t n) {
  return rows >= 0 && rows <= (int64_t(1) << 40) && (k_out == 1 || k_out == 2 || k_out == 3 || k_out == 4 ||
                                                      k_out == 6 || k_out == 8) &&
         n >= 128 && n % 128 == 0 && 1024 % n == 0;
}

int64_t vss_output_backward_direct_chunks(int64_t rows, int32_t k_out, int32_t n) {
  if (!output_direct_ok(rows, k_out, n)) return -1;
  return rows == 0 ? 0 : vgemm::direct_plan(rows, n).blocks;
}

int vss_output_backward_direct(void* stream, int64_t rows, int32_t k_out, int32_t n, const float* g_out,
                               const float* w_out, const float* y, float* grad_in, float* bias_partial,
                               float* wgrad_partial) {
  if (!output_direct_ok(rows, k_out, n) || !g_out || !w_out || misaligned(y) || misaligned(grad_in) ||
      misaligned(bias_partial) || misaligned(wgrad_partial))
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const vgemm::SmallPlan sp = vgemm::direct_plan(rows, n);
  const dim3 grid((unsigned)sp.blocks), block(vgemm::kDirThreads);
  switch (k_out) {
#define VSS_OBD_CASE(KO)                                                                                          \
  case KO:                                                                                                        \
    hipLaunchKernelGGL((vgemm::output_backward_direct_kernel<KO>), grid, block, 0, (hipStream_t)stream, rows, n,  \
                       g_out, w_out, y, grad_in, bias_partial, sp.rows_per_block, wgrad_partial);                 \
    break;
    VSS_OBD_CASE(1)
    VSS_OBD_CASE(2)
    VSS_OBD_CASE(3)
    VSS_OBD_CASE(4)
    VSS_OBD_CASE(6)
    VSS_OBD_CASE(8)
#undef VSS_OBD_CASE
    default:
      return VSS_E_ARG;
  }
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
