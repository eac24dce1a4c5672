// vss_gemm_x6.hip — the PPO update's GEMMs in fp32 arithmetic on the bf16 matrix cores (gfx950).
//
// SURVEY §8 A13 (ppo_continuous_action_isaacgym.py:306-353): one update back-propagates 32 minibatches
// of 2,097,152 rows through both 5-layer MLPs (ppo…:104-125), 4.3e14 FLOP, 94 % of it in the hidden
// layers' GEMMs.  gfx950's fp32-input MFMA (v_mfma_f32_32x32x2_f32, vss_update.hip) peaks at 157 TF;
// its bf16 MFMA at 16x that.  This file computes the same fp32 products on the bf16 pipe:
//
//   every fp32 operand is split EXACTLY into three bf16 parts, v = hi + mid + lo:
//     hi  = bf16_rne(v),  r1 = v - hi          (exact in fp32: r1 has <= 16 significant bits)
//     mid = bf16_rne(r1), lo = r1 - mid        (exact: lo has <= 8 significant bits, a bf16)
//   so |mid| <= 2^-8 |v|, |lo| <= 2^-16 |v| (relative to v's exponent), and
//     a b = ah bh + (ah bm + am bh) + (ah bl + am bm + al bh) + [am bl + al bm + al bl]
//   The six products before the bracket are bf16 x bf16 products (exact in the fp32 accumulator);
//   the bracket is below 2^-23 |a||b| (about one fp32 ulp of the product) and is dropped.  Each K step
//   of 32 runs the six products as six v_mfma_f32_16x16x32_bf16, smallest first, into one fp32
//   accumulator.  Error vs an fp64 reference: that of an fp32 GEMM (tests/test_gemm_x6.py measures it
//   beside the fp32 MFMA kernels and hipBLASLt's fp32 GEMM).
//
// Orientation: the kernel computes D[i][j] = sum_t P[i][t] Q[j][t] and stores D transposed,
// out[j][i] (i contiguous): an accumulator of v_mfma_f32_16x16x32_bf16 holds rows 4 (lane >> 4) ..
// +3 of column lane & 15, i.e. four consecutive i of one j, one 16-B store.
//   forward   (vss_linear_tanh_bf16x6):          i = output feature (P = W, (n, k)), j = row (Q = x)
//   backward  (vss_linear_tanh_backward_bf16x6): i = feature (P = W_next^T, (n, k_next)), j = row (Q = grad_next)
//   weight gradient (vss_weight_grad_bf16x6):     i = input feature (P = x^T), j = output feature
//                                                 (Q = grad^T), contraction over the rows, split in S parts
// P and Q are staged from global memory through registers (fp32), split, and written into a
// double-buffered LDS image [plane][k group of 8][row][8 bf16] (lane groups chosen so that the
// staging writes and the fragment reads are conflict-free).  "Row" operands (forward / backward) are
// K-contiguous in global memory (2 x 16-B loads per 8-wide group); "transposed" operands (weight
// gradient) have the contraction as their ROW index in global memory, and each lane gathers a group
// of 8 rows of one column (8 dword loads, each 256 B contiguous across the wave).
//
// Block: BI x BJ = 128 x 256 outputs, 8 waves as 2 (i) x 4 (j), each 64 x 64 = 4 x 4 MFMA tiles; one
// block per CU (147 KB LDS), persistent over the work items with one flat K pipeline (two register
// sets: a K tile's loads are issued two MFMA phases before the LDS write that consumes them), and the
// XCD-aware slot map of vss_update.hip (the i tiles of a row band run together on one XCD).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/vss.h"
#include "vss_loss_row.h"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_gemm_x6.hip targets gfx950 (CDNA4) only: v_mfma_f32_16x16x32_bf16, v_cvt_pk_bf16_f32"
#endif


namespace vx6 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef short i16x4 __attribute__((ext_vector_type(4)));

enum { EPI_TANH = 0, EPI_DTANH = 1, EPI_TANH_OUT = 2, EPI_WGRAD = 3, EPI_LOSS_A = 4, EPI_LOSS_C = 5 };
enum { ST_ROW = 0, ST_TR = 1, ST_DMA = 2, ST_TR2 = 3, ST_KROW = 4 };

constexpr int KT = 32;  // K tile = one v_mfma_f32_16x16x32_bf16 step
// EPI_DTANH: y row groups requested at the item's last K-tile pair (the rest at the epilogue's start);
// two groups there spill and run 2-5 % slower (profiles/r03z_gemm_x6_colsum.log)
constexpr int kYPre = 1;

// tanh as vss_update.hip's tanh_f32 (odd polynomial below 0.3, exp2 form above)
__device__ __forceinline__ float tanh_f32(float z) {
  const float a = fabsf(z), s = z * z;
  const float poly = z + z * s * (-0.333333343f + s * (0.133333340f + s * (-0.0539682545f + s * 0.0218694885f)));
  const float t = __builtin_amdgcn_exp2f(-2.8853900817779268f * a);
  const float ex = copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), z);
  return a < 0.3f ? poly : ex;
}

// two floats -> packed bf16 (round to nearest even, v_cvt_pk_bf16_f32), element 0 in the low half
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// the exact three-way split of 8 floats (one k group) into hi / mid / lo bf16x8
__device__ __forceinline__ void split8(const float (&v)[8], u32x4& hi, u32x4& mid, u32x4& lo) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    const uint32_t h = pk_bf16(a, b);
    const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xFFFF0000u);
    const uint32_t m = pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(m << 16), sb = rb - __uint_as_float(m & 0xFFFF0000u);
    // sa, sb have <= 8 significant bits: their upper halves are exact bf16
    const uint32_t l = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
    hi[p] = h;
    mid[p] = m;
    lo[p] = l;
  }
}

// LDS image of an R-row operand tile for one K tile: [plane 3][group 4][R][8 bf16]; 16 B per (row,
// group), group stride R * 16 B (a multiple of 256).  Conflict-free on gfx950's lane groups
// (MI355X_MICROARCH.md §LDS): a fragment read's 16-lane groups ({0-3, 12-15, 20-27}, ...) take rows
// fr of group fg at fg * GS + 16 fr -- 16 distinct 16-B slots of the 256-B bank row -- and a staging
// write's 8-lane groups write 8 consecutive rows of one group (128 contiguous bytes).  (A 64-B group
// pad measured 705 M bank-conflict cycles per 10 launches: 2-way reads and writes.)
template <int R>
struct Img {
  static constexpr int GS = R * 16;  // bytes
  static constexpr int PS = 4 * GS;
  static constexpr int BYTES = 3 * PS;
};

// ST_KROW image of an R-column operand whose contraction index is its ROW in global memory (the weight
// gradient's x and grad, (rows, R)): [plane 3][R / 128 sub-tiles][32 contraction rows][128 bf16], i.e.
// the global layout, 256 B per row, with the 16-B chunks of row r XOR-swizzled by
// kswz(r) = ((r & 3) << 2) | ((r >> 2) & 3).  The staging writes whole rows (16 B per lane, an 8-lane
// write group = 8 chunks of one row: conflict-free), and the MFMA fragment -- 8 consecutive contraction
// rows of one feature -- is read TRANSPOSED with two ds_read_b64_tr_b16 (rows 8 fg + q and 8 fg + 4 + q,
// MI355X / cdna_hip_programming.md T10): each 32-lane half then touches 16 distinct 16-B slots of the
// 256-B bank row (layout (b) of T10).  No register transpose and only 16-B global loads: the ST_TR /
// ST_TR2 staging it replaces gathered each k group of a column with 8 dword loads per lane.
__device__ __forceinline__ int kswz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
template <int R>
struct KImg {
  static constexpr int SUB = 32 * 256;
  static constexpr int PS = (R / 128) * SUB;
  static_assert(R % 128 == 0 && 3 * PS == Img<R>::BYTES, "ST_KROW: whole 128-feature sub-tiles, same bytes as Img");
};
// byte offset (within one plane of a KImg) of the half-h transposed read of the fragment of features
// i0 .. i0 + 15 (i0 % 16 == 0): lane 4q + p of 16-lane group fg addresses contraction row 8 fg + 4 h + q,
// features i0 + 4p .. + 3; lane fr of the group receives feature i0 + fr, rows in elements 0..3
__device__ __forceinline__ int kfrag_off(int i0, int lane, int h) {
  const int q = (lane >> 2) & 3, p = lane & 3, row = 8 * (lane >> 4) + 4 * h + q;
  const int c = ((i0 & 127) >> 3) + (p >> 1);
  return (i0 >> 7) * (32 * 256) + row * 256 + 16 * (c ^ kswz(row)) + 8 * (p & 1);
}
__device__ __forceinline__ u32x4 tr_frag(const char* lds_at_a, const char* lds_at_b) {
  typedef __attribute__((address_space(3))) i16x4* lp;
  const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(lds_at_a));
  const i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(lds_at_b));
  const uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  return (u32x4){ua.x, ua.y, ub.x, ub.y};
}

template <int BI_, int BJ_, int WI_, int WJ_>
struct Cfg {
  static constexpr int BI = BI_, BJ = BJ_, WI = WI_, WJ = WJ_;
  static constexpr int THREADS = 64 * WI * WJ;
  static constexpr int WTI = BI / WI, WTJ = BJ / WJ;  // one wave's output extent
  static constexpr int TI = WTI / 16, TJ = WTJ / 16;  // MFMA tiles per wave
  static constexpr int PI = BI * 4 / THREADS, PJ = BJ * 4 / THREADS;  // (row, group) pairs per thread
  static constexpr int BUF = Img<BI>::BYTES + Img<BJ>::BYTES;
  static constexpr int LDS = 2 * BUF;
  static_assert(PI * THREADS == BI * 4 && PJ * THREADS == BJ * 4, "staging pairs must tile the block");
  static_assert(WTI == 64, "a wave's i extent is one 64-feature slice (EPI_TANH_OUT)");
  static constexpr int BPC = 2 * LDS <= 160 * 1024 ? 2 : 1;  // blocks per CU (LDS-limited)
  static_assert(LDS <= 160 * 1024, "the LDS image must fit a CU");
};
using CfgA = Cfg<128, 256, 2, 4>;
// forward / backward with n % 256 == 0 (every layer of the Agent): 256 features x 128 rows, 4 x 2
// waves.  Against CfgA the activation tile each block stages through registers and splits is half
// as large and is shared by half as many blocks (ni = n / 256), while the weight tile, twice as
// large, still arrives by LDS-DMA: forward 8-10 %, backward 1-2 % faster, the same bits
// (profiles/r03z_gemm_x6_fb256.log)
using CfgB = Cfg<256, 128, 4, 2>;

struct Args {
  int32_t ni, nj;          // i tiles, j tiles (of BI, BJ)
  int64_t kpairs;          // K-tile pairs of the whole contraction
  int32_t items;           // work items = ni * nj * splits
  int32_t splits;          // contraction parts (EPI_WGRAD; 1 otherwise): part s takes K-tile pairs
                           // [s kpairs / splits, (s + 1) kpairs / splits)
  int64_t ldp, ldq;        // row strides (floats) of P and Q in global memory
  const void* p;           // ST_TR: (K, I), i.e. rows of the contraction; ST_DMA: the tile-ordered
                           // LDS images of the (I, K) weight's bf16 planes (split_image_kernel)
  const float* q;          // ST_ROW: (J, K);      ST_TR: (K, J)
  int64_t ldo;             // output row stride (floats): out[j][i]
  float* out;              // (J, I) (EPI_WGRAD: (splits, J, I))
  const float* bias;       // EPI_TANH*: (I)
  const float* y;          // EPI_DTANH: (J, I) the tanh output the gradient passes through
  float* partial;          // EPI_DTANH: (grid / ni, I) column sums of out
  const float* w_out;      // EPI_TANH_OUT / EPI_LOSS_*: (KO, I)
  float* out_part;         // EPI_TANH_OUT: (I / 64, J, KO)
  // EPI_LOSS_A / EPI_LOSS_C: the last hidden layer, the output layer and the minibatch loss of
  // ppo…:318-349 (the actor's policy terms / the critic's value terms) folded into one epilogue; out receives
  // the hidden layer's pre-activation gradient gz = (g_out W_out) (1 - y^2), never y
  const float* b_out;      // (KO) the output layer's bias
  const float* l_act;      // actor: the actions (rows, KO)
  const float* l_logp;     // actor: the rollout log-probs (rows)
  const float* l_adv;      // actor: the RAW advantages (rows), normalised from adv_part when given
  const double* adv_part;  // actor: (adv_nparts, 2) fp64 (sum, sum of squares) parts, or NULL
  int32_t adv_nparts;
  double adv_count;
  const float* logstd;     // actor: (KO)
  const float* l_ret;      // critic: returns (rows)
  const float* l_val;      // critic: rollout values (rows), read with clip_vloss
  float clip, clip_lo, clip_hi, vf_coef, inv_n;
  int32_t clip_vloss;
  int64_t rows_real;       // rows of the minibatch (the rest are padding: zero gradient, no loss term)
  float* part_cs;          // (grid, I) the block's column sums of gz (the hidden layer's bias gradient)
  float* part_dwo;         // (grid, KO, I) the block's g_out^T y (the output layer's weight gradient)
  float* part_stats;       // (grid, 32) the block's loss sums (kLossStats layout)
};

// EPI_LOSS_*: per-block loss sums (vss_loss_row.h kBlockStats layout)
constexpr int kLossStats = vlossrow::kBlockStats;

// one thread's register-staged operands of one K tile: NP groups of 8 raw fp32 values
template <int NP>
struct Stage {
  u32x4 v[NP][2];
};

template <int MODE, int R, int NP, class C>
__device__ __forceinline__ void load_op(u32x4 (*dst)[2], const void* base_, int64_t ld, int64_t k0) {
  const int t = threadIdx.x;
  if constexpr (MODE == ST_TR2) {
    // ST_TR with two adjacent columns (image rows) per lane: one 8-B load per contraction row, half
    // the load instructions for the same bytes (a wave reads 512 contiguous bytes of a row); weight
    // gradient 1-2 % faster (profiles/r03zz_gemm_x6_tr2.log)
    static_assert(NP == 2 && (R / 2) * 4 == C::THREADS, "ST_TR2: one column pair x 4 k groups per thread");
    const int c2 = t % (R / 2), g = t / (R / 2);
    const float* src = static_cast<const float*>(base_) + (k0 + 8 * g) * ld + 2 * c2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float2 x = *reinterpret_cast<const float2*>(src + e * ld);
      dst[0][e >> 2][e & 3] = __float_as_uint(x.x);
      dst[1][e >> 2][e & 3] = __float_as_uint(x.y);
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int pr = t + C::THREADS * u;
    if constexpr (MODE == ST_KROW) {
      // 8 consecutive features of one contraction row: a wave reads R / 8 lanes x 32 B per row
      const int row = pr / (R / 8), cc = pr % (R / 8);
      const float* src = static_cast<const float*>(base_) + (k0 + row) * ld + 8 * cc;
      dst[u][0] = *reinterpret_cast<const u32x4*>(src);
      dst[u][1] = *reinterpret_cast<const u32x4*>(src + 4);
    } else if constexpr (MODE == ST_ROW) {
      const int g = (pr >> 3) & 3, row = (pr & 7) | ((pr >> 5) << 3);
      const float* src = static_cast<const float*>(base_) + (int64_t)row * ld + k0 + 8 * g;
      dst[u][0] = *reinterpret_cast<const u32x4*>(src);
      dst[u][1] = *reinterpret_cast<const u32x4*>(src + 4);
    } else {
      const int row = pr % R, g = pr / R;
      const float* src = static_cast<const float*>(base_) + (k0 + 8 * g) * ld + row;
#pragma unroll
      for (int e = 0; e < 8; ++e) dst[u][e >> 2][e & 3] = __float_as_uint(src[e * ld]);
    }
  }
}

template <int MODE, int R, int NP, class C>
__device__ __forceinline__ void write_op(const u32x4 (*src)[2], char* img) {
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int pr = t + C::THREADS * u;
    int g, row;
    if constexpr (MODE == ST_TR) {
      row = pr % R;
      g = pr / R;
    } else if constexpr (MODE == ST_TR2) {
      // the lane's column pair: image rows 2 c2 and 2 c2 + 1.  An 8-lane write group then covers
      // 4 row residues mod 8 (a 2-way bank conflict); swapping the pair's order in half the lanes
      // removes it but its selects cost more than the conflict (1-3 % slower, r03zz_gemm_x6_tr2.log)
      row = 2 * (t % (R / 2)) + u;
      g = t / (R / 2);
    } else {
      g = (pr >> 3) & 3;  // lanes 8 q .. 8 q + 7: 8 consecutive rows of one group (one write lane group)
      row = (pr & 7) | ((pr >> 5) << 3);
    }
    u32x4 hi, mid, lo;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = __uint_as_float(src[u][e >> 2][e & 3]);
    split8(v, hi, mid, lo);
    char* d;
    int ps;
    if constexpr (MODE == ST_KROW) {
      const int kr = pr / (R / 8), cc = pr % (R / 8);
      d = img + (cc >> 4) * KImg<R>::SUB + kr * 256 + 16 * ((cc & 15) ^ kswz(kr));
      ps = KImg<R>::PS;
    } else {
      d = img + g * Img<R>::GS + row * 16;
      ps = Img<R>::PS;
    }
    *reinterpret_cast<u32x4*>(d) = hi;
    *reinterpret_cast<u32x4*>(d + ps) = mid;
    *reinterpret_cast<u32x4*>(d + 2 * ps) = lo;
  }
}

// W (n, K) fp32 -> the LDS images of its three bf16 planes, tile by tile (ST_DMA): for i tile it
// (128 rows) and K tile kt, [plane][k group g][row r][8 bf16] of W[128 it + r][32 kt + 8 g + e] --
// exactly the bytes of the GEMM's P image, so each wave copies its slice with global_load_lds_dwordx4
// (1 KB per wave instruction, contiguous in global memory and LDS)
template <int R>
__global__ __launch_bounds__(256) void split_image_kernel(const float* __restrict__ w, int64_t n, int64_t k,
                                                          uint16_t* __restrict__ img) {
  const int64_t ktn = k / KT, units = n * k / 8;
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (it, kt, g, r), r fastest
  if (u >= units) return;
  const int r = (int)(u % R), g = (int)((u / R) % 4);
  const int64_t kt = (u / (4 * R)) % ktn, it = u / (4 * R * ktn);
  const float* src = w + (it * R + r) * k + kt * KT + 8 * g;
  const u32x4 a = *reinterpret_cast<const u32x4*>(src), b = *reinterpret_cast<const u32x4*>(src + 4);
  float v[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = __uint_as_float(a[e]);
    v[4 + e] = __uint_as_float(b[e]);
  }
  u32x4 hi, mid, lo;
  split8(v, hi, mid, lo);
  uint16_t* d = img + (it * ktn + kt) * (3 * 4 * R * 8) + (g * R + r) * 8;
  *reinterpret_cast<u32x4*>(d) = hi;
  *reinterpret_cast<u32x4*>(d + 4 * R * 8) = mid;
  *reinterpret_cast<u32x4*>(d + 2 * 4 * R * 8) = lo;
}

// several weights' plane images in one launch (vss_weight_planes_bf16x6): job blockIdx.y, the same image
// bytes as split_image_kernel<r>; `trans` = the job's fp32 weight is stored (k, n), i.e. the image is
// of its transpose (the backward's W_next^T, without a transposed copy)
struct PlaneJob {
  const float* w;
  uint16_t* img;
  int64_t n, k;
  int32_t trans, r;
};
constexpr int kMaxPlaneJobs = 16;  // both MLPs of the Agent: 2 x 6
struct PlaneJobs {
  PlaneJob j[kMaxPlaneJobs];
};

__global__ __launch_bounds__(256) void plane_images_kernel(PlaneJobs jobs) {
  const PlaneJob& J = jobs.j[blockIdx.y];
  const int64_t ktn = J.k / KT, units = J.n * J.k / 8;
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (it, kt, g, r), r fastest
  if (u >= units) return;
  const int R = J.r;
  const int r = (int)(u % R), g = (int)((u / R) % 4);
  const int64_t kt = (u / (4 * R)) % ktn, it = u / (4 * R * ktn);
  const int64_t row = it * R + r, col = kt * KT + 8 * g;  // element (row, col .. col + 7) of the (n, k) operand
  float v[8];
  if (J.trans) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = J.w[(col + e) * J.n + row];  // lanes r: consecutive words of one row of w
  } else {
    const u32x4 a = *reinterpret_cast<const u32x4*>(J.w + row * J.k + col);
    const u32x4 b = *reinterpret_cast<const u32x4*>(J.w + row * J.k + col + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = __uint_as_float(a[e]);
      v[4 + e] = __uint_as_float(b[e]);
    }
  }
  u32x4 hi, mid, lo;
  split8(v, hi, mid, lo);
  uint16_t* d = J.img + (it * ktn + kt) * (3 * 4 * (int64_t)R * 8) + ((int64_t)g * R + r) * 8;
  *reinterpret_cast<u32x4*>(d) = hi;
  *reinterpret_cast<u32x4*>(d + 4 * R * 8) = mid;
  *reinterpret_cast<u32x4*>(d + 2 * 4 * R * 8) = lo;
}

// sum over the 16 lanes of a DPP row (as vss_update.hip row16_sum)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<0xB1>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x140>(v);
  return v;
}
// v summed over the four rows of 16 lanes (an MFMA output column's k groups fg): v + v of lane ^ 16, then +
// that of lane ^ 32 -- the pairs and the bits of __shfl_xor 16 / 32, by v_permlane16_swap / v_permlane32_swap
// instead of two LDS round trips
__device__ __forceinline__ float kgroup_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// sum over the 64 lanes, every lane getting the same bits (each step adds a pair in an order-free way)
__device__ __forceinline__ float wave64_sum(float v) { return kgroup_sum(row16_sum(v)); }
// m's bit for this lane ? b : a, as one v_cndmask_b32 (written as C selects over an array, the tree below is
// turned into a scratch-indexed load)
__device__ __forceinline__ float lane_sel(uint64_t m, float a, float b) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}
// t[k] for k = the lane's index (0 .. 15) by a select tree on its bits (no exec-mask branch): after row16_sum
// every lane of a row holds every sum, so lane k can write the k-th one
__device__ __forceinline__ float pick16(const float (&t)[16], int k) {
  const uint64_t m0 = __builtin_amdgcn_ballot_w64(k & 1), m1 = __builtin_amdgcn_ballot_w64(k & 2),
                 m2 = __builtin_amdgcn_ballot_w64(k & 4), m3 = __builtin_amdgcn_ballot_w64(k & 8);
  float a[8], b[4], c[2];
#pragma unroll
  for (int m = 0; m < 8; ++m) a[m] = lane_sel(m0, t[2 * m], t[2 * m + 1]);
#pragma unroll
  for (int m = 0; m < 4; ++m) b[m] = lane_sel(m1, a[2 * m], a[2 * m + 1]);
#pragma unroll
  for (int m = 0; m < 2; ++m) c[m] = lane_sel(m2, b[2 * m], b[2 * m + 1]);
  return lane_sel(m3, c[0], c[1]);
}

template <int EPI, int SP, int SQ, class C, int KO = 0>
__global__ __launch_bounds__(C::THREADS, C::BPC) void gemm_x6_kernel(Args a) {
  constexpr int BI = C::BI, BJ = C::BJ, TI = C::TI, TJ = C::TJ, PJ = C::PJ;
  // ST_DMA: the weight operand's image is copied global -> LDS by the waves' global_load_lds (3 KB per
  // wave per K tile), only the activations go through registers
  constexpr bool PDMA = SP == ST_DMA;
  constexpr int PI = PDMA ? 0 : C::PI;
  constexpr int NQ = Img<BI>::BYTES / (C::THREADS / 64) / 1024;  // 1-KB DMA slices per wave per K tile
  static_assert(!PDMA || NQ * (C::THREADS / 64) * 1024 == Img<BI>::BYTES, "DMA slices: whole KB per wave");
  // EPI_DTANH: (WJ, BI) column sums, accumulated item by item
  constexpr bool LOSS = EPI == EPI_LOSS_A || EPI == EPI_LOSS_C;
  // EPI_LOSS_*: bias | W_out | the output parts / row gradients (WI x BJ x KO) | column sums (WJ x BI) |
  // g_out^T y (WJ x KO x BI) | loss sums of waves 0, 1 (2 x 32) | advantage mean, std
  constexpr int E_P = BI + KO * 256, E_CS = E_P + C::WI * BJ * KO, E_DW = E_CS + C::WJ * BI,
                E_ST = E_DW + C::WJ * KO * BI, E_AD = E_ST + 2 * kLossStats;
  constexpr int EPI_FLOATS = LOSS ? E_AD + 2
                                  : (EPI == EPI_TANH_OUT ? KO * 256 + BI
                                                         : (EPI == EPI_WGRAD ? 1 : (EPI == EPI_DTANH ? C::WJ * BI : BI)));
  static_assert(!LOSS || (BI == 256 && KO >= 1 && KO <= 2), "EPI_LOSS_*: whole 256-feature rows, 1 or 2 outputs");
  // one LDS object (a second __shared__ array beside a global_load_lds target can make hipcc wait
  // vmcnt(0) before the k-steps' LDS reads, cdna_hip_programming.md §5)
  __shared__ __attribute__((aligned(16))) char lds[C::LDS + EPI_FLOATS * 4];
  float* epi_lds = reinterpret_cast<float*>(lds + C::LDS);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv / C::WJ, wj = wv % C::WJ;
  const int G = gridDim.x;
  const int slot = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (slot >= a.items) return;
  const int per_split = a.ni * a.nj;

  // work item w -> (split, j tile, i tile); j-band major so the ni i tiles of a band are consecutive
  auto item_ij = [&](int w, int& it, int& jt, int& sp) {
    sp = w / per_split;
    const int r = w % per_split;
    jt = r / a.ni;
    it = r % a.ni;
  };

  // per-block constants of a fixed i tile (the host makes G a multiple of 8 ni for EPI != EPI_WGRAD)
  int it0, jt0, sp0;
  item_ij(slot, it0, jt0, sp0);
  if constexpr (EPI != EPI_WGRAD) {
    for (int i = tid; i < (EPI == EPI_DTANH ? EPI_FLOATS : BI); i += C::THREADS)
      epi_lds[i] = EPI == EPI_DTANH ? 0.f : a.bias[it0 * BI + i];
    if constexpr (EPI == EPI_TANH_OUT || LOSS)
      for (int i = tid; i < KO * 256; i += C::THREADS) epi_lds[BI + i] = a.w_out[i];
    if constexpr (LOSS) {
      for (int i = E_CS + tid; i < E_AD; i += C::THREADS) epi_lds[i] = 0.f;
      if (EPI == EPI_LOSS_A && a.adv_part && wv == 0) {
        // the advantages' mean and std from the fp64 parts (vss_loss.hip adv_moments' order)
        double s0 = 0.0, q0 = 0.0;
        for (int i = lane; i < a.adv_nparts; i += 64) {
          s0 += a.adv_part[2 * i];
          q0 += a.adv_part[2 * i + 1];
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
          s0 += __shfl_xor(s0, m);
          q0 += __shfl_xor(q0, m);
        }
        if (lane == 0) {
          const double n = a.adv_count, m = s0 / n;
          double var = (q0 - n * m * m) / (n - 1.0);
          var = var > 0.0 ? var : 0.0;
          epi_lds[E_AD] = (float)m;
          epi_lds[E_AD + 1] = (float)sqrt(var);
        }
      }
    }
  }

  // fetch cursor over the flat sequence of (item, k tile)
  int f_item = slot, f_kt = 0;
  const char* fp;
  const char* fq;
  // first K tile of contraction part sp (parts differ by at most one K-tile pair)
  auto kt_lo = [&](int sp) -> int64_t {
    if constexpr (EPI == EPI_WGRAD) return 2 * ((int64_t)sp * a.kpairs / a.splits);
    return sp == 0 ? 0 : 2 * a.kpairs;  // one part
  };
  int64_t fk0 = 0;  // contraction offset of the fetched item (EPI_WGRAD part)
  int f_kn = 0;     // its K tiles
  auto point = [&](int w) {
    int it, jt, sp;
    item_ij(w, it, jt, sp);
    fk0 = kt_lo(sp) * KT;
    f_kn = (int)(kt_lo(sp + 1) - kt_lo(sp));
    if constexpr (SP == ST_TR || SP == ST_KROW) fp = static_cast<const char*>(a.p) + (int64_t)it * BI * 4;
    else fp = static_cast<const char*>(a.p);  // ST_DMA: addressed by dma_p
    if constexpr (SQ == ST_TR || SQ == ST_TR2 || SQ == ST_KROW)
      fq = reinterpret_cast<const char*>(a.q) + (int64_t)jt * BJ * 4;
    else fq = reinterpret_cast<const char*>(a.q) + (int64_t)jt * BJ * a.ldq * 4;
  };
  point(f_item);
  auto gload = [&](Stage<PI + PJ>& s) {
    const int64_t k0 = fk0 + (int64_t)f_kt * KT;
    if constexpr (!PDMA) load_op<SP, BI, PI, C>(s.v, fp, a.ldp, k0);
    load_op<SQ, BJ, PJ, C>(s.v + PI, fq, a.ldq, k0);
    if (++f_kt >= f_kn) {
      if (f_item + G < a.items) {
        f_kt = 0;
        f_item += G;
        point(f_item);
      } else {
        f_kt = f_kn - 1;  // past the last item: re-load its last K tile (in bounds, never used)
      }
    }
  };
  auto swrite = [&](const Stage<PI + PJ>& s, int buf) {
    char* base = lds + buf * C::BUF;
    if constexpr (!PDMA) write_op<SP, BI, PI, C>(s.v, base);
    write_op<SQ, BJ, PJ, C>(s.v + PI, base + Img<BI>::BYTES);
  };
  // ST_DMA: K tile kt of the block's i tile it0 -> the P image of LDS buffer buf
  auto dma_p = [&](int64_t kt, int buf) {
    if constexpr (PDMA) {
      const int64_t off = ((int64_t)it0 * (2 * a.kpairs) + kt) * Img<BI>::BYTES;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int slice = (wv * NQ + q) * 1024;
        // (C-style casts: the builtin takes a global and an LDS address-space pointer)
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void*)(static_cast<const char*>(a.p) + off + slice + lane * 16),
            (__attribute__((address_space(3))) void*)(lds + buf * C::BUF + slice), 16, 0, 0);
      }
    }
  };

  f32x4 acc[TI][TJ];
  const int fr = lane & 15, fg = lane >> 4;  // fragment row, k group
  // the K tile in LDS buffer buf; `between` runs after its fragment reads are issued and before its
  // MFMAs (ST_DMA: the next P image's global_load_lds, kept behind the reads so that hipcc's
  // LDS-alias wait for the DMA does not land before them)
  auto mfma_tile = [&](int buf, auto&& between) {
    const char* pb = lds + buf * C::BUF + fg * Img<BI>::GS + (wi * C::WTI + fr) * 16;
    const char* qb = lds + buf * C::BUF + Img<BI>::BYTES + fg * Img<BJ>::GS + (wj * C::WTJ + fr) * 16;
    u32x4 pf[3][TI], qf[3][TJ];
    const char* pk = lds + buf * C::BUF;                    // ST_KROW images: plane 0 of P
    const char* qk = lds + buf * C::BUF + Img<BI>::BYTES;  // and of Q
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if constexpr (SP == ST_KROW) {
          const int i0 = wi * C::WTI + 16 * i;
          pf[pl][i] = tr_frag(pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 0), pk + pl * KImg<BI>::PS + kfrag_off(i0, lane, 1));
        } else {
          pf[pl][i] = *reinterpret_cast<const u32x4*>(pb + pl * Img<BI>::PS + i * 256);
        }
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        if constexpr (SQ == ST_KROW) {
          const int j0 = wj * C::WTJ + 16 * j;
          qf[pl][j] = tr_frag(qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 0), qk + pl * KImg<BJ>::PS + kfrag_off(j0, lane, 1));
        } else {
          qf[pl][j] = *reinterpret_cast<const u32x4*>(qb + pl * Img<BJ>::PS + j * 256);
        }
      }
    }
    if constexpr (PDMA) {
      __builtin_amdgcn_sched_barrier(0);
      between();
      __builtin_amdgcn_sched_barrier(0);
    }
    // the six products, smallest first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
    for (int x = 0; x < 6; ++x)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pf[PP[x]][i]),
                                                              __builtin_bit_cast(bf16x8, qf[QP[x]][j]), acc[i][j], 0, 0, 0);
  };

  // EPI_LOSS_*: the item's epilogue in three phases separated by barriers.  (1) y = tanh(acc + b) kept in
  // the accumulators, the wave's 64-feature slice of each row's output-layer sums into LDS; (2) one thread
  // per row: the output (4 slices in order, then the bias), that row's loss terms and its gradient g_out
  // (zero for padding rows), the terms summed per wave into LDS; (3) every lane: gz = (g_out W_out)
  // (1 - y^2) stored for its rows and features, and the item's column sums of gz and g_out^T y added to
  // per-(wave row, feature) slots (one lane per slot).
  auto loss_epilogue = [&](f32x4 (&ac)[TI][TJ], int it, int jt) __attribute__((always_inline)) {
    if constexpr (LOSS) {
      const int ib = it * BI + wi * C::WTI;
      // phase 2's inputs, requested before phase 1 (waves 0 and 1: one thread per row) so that their latency
      // hides behind phase 1's tanh and output sums instead of stalling the two waves after its barrier
      const int64_t grow = (int64_t)jt * BJ + tid;
      const bool row_real = tid < BJ && grow < a.rows_real;
      float in_x[KO], in_b[KO], in_ls[KO], in_a = 0.f, in_l = 0.f;
#pragma unroll
      for (int o = 0; o < KO; ++o) in_x[o] = in_b[o] = in_ls[o] = 0.f;
      if (tid < BJ) {
#pragma unroll
        for (int o = 0; o < KO; ++o) {
          in_b[o] = a.b_out[o];
          if constexpr (EPI == EPI_LOSS_A) in_ls[o] = a.logstd[o];
        }
        if (row_real) {
          if constexpr (EPI == EPI_LOSS_A) {
#pragma unroll
            for (int o = 0; o < KO; ++o) in_x[o] = a.l_act[grow * KO + o];
            in_a = a.l_adv[grow];
            in_l = a.l_logp[grow];
          } else {
            in_a = a.l_ret[grow];
            in_l = a.clip_vloss ? a.l_val[grow] : 0.f;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int rl = wj * C::WTJ + 16 * j + fr;  // row within the item
        float od[KO];
#pragma unroll
        for (int o = 0; o < KO; ++o) od[o] = 0.f;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int il = wi * C::WTI + 16 * i + 4 * fg;
          f32x4 v = ac[i][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + epi_lds[il + r]);
          ac[i][j] = v;
#pragma unroll
          for (int o = 0; o < KO; ++o) {
            const float* wo = epi_lds + BI + o * 256 + ib + 16 * i + 4 * fg;
            float d = v[0] * wo[0];
            d = fmaf(v[1], wo[1], d);
            d = fmaf(v[2], wo[2], d);
            d = fmaf(v[3], wo[3], d);
            od[o] += d;
          }
        }
#pragma unroll
        for (int o = 0; o < KO; ++o) {
          const float d = kgroup_sum(od[o]);
          if (fg == 0) epi_lds[E_P + (wi * BJ + rl) * KO + o] = d;
        }
      }
      __syncthreads();
      if (tid < BJ) {  // waves 0 and 1 whole: one thread per row of the item
        float outv[KO], g[KO], t[kLossStats > 0 ? 5 + 2 * KO : 1];
#pragma unroll
        for (int o = 0; o < KO; ++o) {
          float d = epi_lds[E_P + tid * KO + o];
#pragma unroll
          for (int q = 1; q < C::WI; ++q) d += epi_lds[E_P + (q * BJ + tid) * KO + o];
          outv[o] = d + in_b[o];
          g[o] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < 5 + 2 * KO; ++k) t[k] = 0.f;
        if (row_real) {
          if constexpr (EPI == EPI_LOSS_A) {
            float var[KO], lsc[KO], gm[KO], lg[KO];
            vlossrow::actor_consts<KO>(in_ls, var, lsc);
            float A = in_a;
            if (a.adv_part) A = (A - epi_lds[E_AD]) / (epi_lds[E_AD + 1] + 1e-8f);
            vlossrow::actor_row<KO>(outv, in_x, in_l, A, var, lsc, a.clip, a.clip_lo, a.clip_hi, a.inv_n, t[0], t[2],
                                    t[3], t[4], gm, lg);
#pragma unroll
            for (int o = 0; o < KO; ++o) {
              g[o] = gm[o];
              t[5 + o] = lg[o];
              t[5 + KO + o] = gm[o];
            }
          } else {
            float gv;
            vlossrow::critic_row(outv[0], in_a, in_l, a.clip_vloss, a.clip, a.vf_coef, a.inv_n, t[1], gv);
            g[0] = gv;
            t[5] = gv;
          }
        }
        // the row gradient over this row's first output part (read above by this thread only)
#pragma unroll
        for (int o = 0; o < KO; ++o) epi_lds[E_P + tid * KO + o] = g[o];
        // the terms summed over the wave (every lane gets every sum), lane k adding the k-th into its slot
        float ts[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) ts[k] = k < 5 + 2 * KO ? wave64_sum(t[k]) : 0.f;
        const float tv = pick16(ts, fr);
        if (lane < 5 + 2 * KO) epi_lds[E_ST + wv * kLossStats + lane] += tv;
      }
      __syncthreads();
      // feature group by feature group (i outer): 4 + 4 KO sums live, not TI times that
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int il = wi * C::WTI + 16 * i + 4 * fg;
        float cs[4] = {0.f, 0.f, 0.f, 0.f}, dw[4][KO];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int o = 0; o < KO; ++o) dw[r][o] = 0.f;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int rl = wj * C::WTJ + 16 * j + fr;
          const int64_t jg = (int64_t)jt * BJ + rl;
          float g[KO];
#pragma unroll
          for (int o = 0; o < KO; ++o) g[o] = epi_lds[E_P + rl * KO + o];
          const f32x4 v = ac[i][j];
          vx6::f32x4 z;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float sg = g[0] * epi_lds[BI + il + r];
#pragma unroll
            for (int o = 1; o < KO; ++o) sg = fmaf(g[o], epi_lds[BI + o * 256 + il + r], sg);
            z[r] = sg * fmaf(-v[r], v[r], 1.0f);
            cs[r] += z[r];
#pragma unroll
            for (int o = 0; o < KO; ++o) dw[r][o] = fmaf(g[o], v[r], dw[r][o]);
          }
          __builtin_nontemporal_store(z, reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ib + 16 * i + 4 * fg));
        }
        // the 4 + 4 KO sums over the 16 rows, lane fr adding the fr-th into its slot: one read-modify-write
        // of distinct words per feature group, not 4 + 4 KO serial ones by lane 0 of each row
        float t[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          t[r] = row16_sum(cs[r]);
#pragma unroll
          for (int o = 0; o < KO; ++o) t[4 + 4 * o + r] = row16_sum(dw[r][o]);
        }
#pragma unroll
        for (int k = 4 + 4 * KO; k < 16; ++k) t[k] = 0.f;
        const float v = pick16(t, fr);
        if (fr < 4 + 4 * KO) {
          const int slot = fr < 4 ? E_CS + wj * BI + il + fr : E_DW + (wj * KO + ((fr - 4) >> 2)) * BI + il + (fr & 3);
          epi_lds[slot] += v;
        }
      }
    }
  };

  Stage<PI + PJ> r0, r1;
  gload(r0);  // K tile 0
  dma_p(0, 0);
  swrite(r0, 0);
  gload(r1);  // K tile 1
  gload(r0);  // K tile 2
  __syncthreads();
  int w = slot;
  for (;;) {
    const int next = w + G;
    const bool has_next = next < a.items;
    int it, jt, sp;
    item_ij(w, it, jt, sp);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // EPI_DTANH: the epilogue's first y row group (tj = 0) is loaded at the start of the item's last
    // K-tile pair, so its HBM latency hides behind that pair's MFMAs instead of stalling the epilogue
    // (a y load issued in the epilogue also waits, by vmcnt's in-order count, for the next item's
    // prefetched K tiles)
    f32x4 ypre[EPI == EPI_DTANH ? kYPre : 1][EPI == EPI_DTANH ? TI : 1];
    const int64_t jy = (int64_t)jt * BJ + wj * C::WTJ + fr;
    const int kn = (int)(kt_lo(sp + 1) - kt_lo(sp));  // this item's K tiles (even)
    for (int kt = 0; kt < kn; kt += 2) {
      if constexpr (EPI == EPI_DTANH) {
        if (kt + 2 >= kn) {
#pragma unroll
          for (int j = 0; j < kYPre; ++j)
#pragma unroll
            for (int i = 0; i < TI; ++i)
              ypre[j][i] = *reinterpret_cast<const f32x4*>(a.y + (jy + 16 * j) * a.ldo + it * BI + wi * C::WTI + 16 * i +
                                                           4 * fg);
        }
      }
      mfma_tile(0, [&] { dma_p(kt + 1, 1); });
      swrite(r1, 1);
      __syncthreads();
      gload(r1);
      mfma_tile(1, [&] {
        if (kt + 2 < kn) dma_p(kt + 2, 0);
        else if (has_next) dma_p(0, 0);  // the next item's first K tile (same i tile, all K tiles)
      });
      swrite(r0, 0);
      __syncthreads();
      gload(r0);
    }

    // epilogue straight from the accumulators: lane holds out[j][i .. i + 3] for
    // i = i0 + 16 ti + 4 fg, j = j0 + 16 tj + fr
    // EPI_DTANH: this item's column sums of the lane's features (16 i + 4 fg + r), over its rows
    float cs[EPI == EPI_DTANH ? TI : 1][4];
#pragma unroll
    for (int i = 0; i < (EPI == EPI_DTANH ? TI : 1); ++i) cs[i][0] = cs[i][1] = cs[i][2] = cs[i][3] = 0.f;
    const int ib = it * BI + wi * C::WTI, jb = jt * BJ + wj * C::WTJ;
    // EPI_DTANH: the other y row groups are all requested before the first group's work, so their
    // latencies overlap one another and that work instead of adding up group by group (the K loop's
    // registers are free here); backward 8-13 % faster than one load per group at its use would be
    // without any y traffic (tools/x6_ablate.py noy, profiles/r03z_epi_ablate.log)
    if constexpr (LOSS) {
      loss_epilogue(acc, it, jt);
      if (!has_next) break;
      w = next;
      continue;
    }
    f32x4 yrest[EPI == EPI_DTANH ? TJ : 1][EPI == EPI_DTANH ? TI : 1];
    if constexpr (EPI == EPI_DTANH) {
#pragma unroll
      for (int j = kYPre; j < TJ; ++j)
#pragma unroll
        for (int i = 0; i < TI; ++i)
          yrest[j][i] = *reinterpret_cast<const f32x4*>(a.y + ((int64_t)jb + 16 * j + fr) * a.ldo + ib + 16 * i + 4 * fg);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int64_t jg = (int64_t)jb + 16 * j + fr;
      float od[KO > 0 ? KO : 1];  // EPI_TANH_OUT: this row's output-layer sums over the wave's features
#pragma unroll
      for (int o = 0; o < (KO > 0 ? KO : 1); ++o) od[o] = 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int il = wi * C::WTI + 16 * i + 4 * fg;  // feature within the block's i tile
        const int ig = it * BI + il;
        f32x4 v = acc[i][j];
        if constexpr (EPI == EPI_TANH || EPI == EPI_TANH_OUT) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + epi_lds[il + r]);
          *reinterpret_cast<f32x4*>(a.out + jg * a.ldo + ig) = v;
          if constexpr (EPI == EPI_TANH_OUT) {
#pragma unroll
            for (int o = 0; o < KO; ++o) {
              const float* wo = epi_lds + BI + o * 256 + ig;
              float d = v[0] * wo[0];
              d = fmaf(v[1], wo[1], d);
              d = fmaf(v[2], wo[2], d);
              d = fmaf(v[3], wo[3], d);
              od[o] += d;
            }
          }
        } else if constexpr (EPI == EPI_DTANH) {
          const f32x4 yv = j < kYPre ? ypre[j < kYPre ? j : 0][i] : yrest[j][i];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = v[r] * fmaf(-yv[r], yv[r], 1.0f);
            cs[i][r] += v[r];
          }
          acc[i][j] = v;  // stored below, two tiles per 128-B line store
        } else {  // EPI_WGRAD: the split's partial
          *reinterpret_cast<f32x4*>(a.out + ((int64_t)sp * a.nj * BJ + jg) * a.ldo + ig) = v;
        }
      }
      if constexpr (EPI == EPI_DTANH) {
        // tiles i and i + 1 of rows jb + 16 j .. + 15 as 128-B line stores: a row rotation by 8 lanes trades the
        // upper 8 rows of tile i for the lower 8 of tile i + 1, so each nontemporal store writes 8 whole 128-B
        // rows (32 consecutive features) instead of 16 half lines: backward 512 <- 256 3.23 vs 3.28 ms, update
        // 2.227 vs 2.236 s (same-box A/B, profiles/r06l_lines_ab.log).  The forwards' plain stores keep one tile
        // per store: as line stores the forward 512 -> 512 ran 2.5 % slower (5.15 vs 5.02 ms, same A/B).
#pragma unroll
        for (int i = 0; i < TI; i += 2) {
          f32x4 lo8, hi8;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xr = dpp_f32<0x128>(acc[i][j][r]), yr = dpp_f32<0x128>(acc[i + 1][j][r]);
            lo8[r] = fr < 8 ? acc[i][j][r] : yr;
            hi8[r] = fr < 8 ? xr : acc[i + 1][j][r];
          }
          const int64_t r0 = (int64_t)jb + 16 * j + (fr & 7);
          const int64_t col = (int64_t)it * BI + wi * C::WTI + 16 * (i + (fr >> 3)) + 4 * fg;
          float* d0 = a.out + r0 * a.ldo + col;
          float* d1 = a.out + (r0 + 8) * a.ldo + col;
          if constexpr (EPI == EPI_DTANH) {
            __builtin_nontemporal_store(lo8, reinterpret_cast<f32x4*>(d0));
            __builtin_nontemporal_store(hi8, reinterpret_cast<f32x4*>(d1));
          } else {
            *reinterpret_cast<f32x4*>(d0) = lo8;
            *reinterpret_cast<f32x4*>(d1) = hi8;
          }
        }
      }
      if constexpr (EPI == EPI_TANH_OUT) {
        // the wave's 64-feature slice of the output layer for row jg: the 4 k groups' lanes
#pragma unroll
        for (int o = 0; o < KO; ++o) {
          const float d = kgroup_sum(od[o]);
          if (fg == 0) a.out_part[(((int64_t)ib >> 6) * (a.nj * BJ) + jg) * KO + o] = d;
        }
      }
    }
    if constexpr (EPI == EPI_DTANH) {
      // the 16 rows (lanes fr) of each k group, added to the wave's (wj, feature) slots: lane fr adds the
      // sum of feature 16 (fr >> 2) + 4 fg + (fr & 3), so the 64 lanes update the wave's 64 slots in one
      // read-modify-write of distinct words (not 16 serial ones by lane 0 of each row)
      static_assert(EPI != EPI_DTANH || TI == 4, "EPI_DTANH column sums: 4 feature tiles per wave");
      float t[16];
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[4 * i + r] = row16_sum(cs[i][r]);
      epi_lds[wj * BI + wi * C::WTI + 16 * (fr >> 2) + 4 * fg + (fr & 3)] += pick16(t, fr);
    }
    if (!has_next) break;
    w = next;
  }

  if constexpr (LOSS) {
    // the WJ waves' slots in order (deterministic); one partial row per block
    __syncthreads();
    for (int f = tid; f < BI; f += C::THREADS) {
      float t = epi_lds[E_CS + f];
#pragma unroll
      for (int m = 1; m < C::WJ; ++m) t += epi_lds[E_CS + m * BI + f];
      a.part_cs[(int64_t)slot * BI + f] = t;
    }
    for (int x = tid; x < KO * BI; x += C::THREADS) {
      const int o = x / BI, f = x - o * BI;
      float t = epi_lds[E_DW + o * BI + f];
#pragma unroll
      for (int m = 1; m < C::WJ; ++m) t += epi_lds[E_DW + (m * KO + o) * BI + f];
      a.part_dwo[((int64_t)slot * KO + o) * BI + f] = t;
    }
    if (tid < kLossStats) a.part_stats[(int64_t)slot * kLossStats + tid] = epi_lds[E_ST + tid] + epi_lds[E_ST + kLossStats + tid];
  }
  if constexpr (EPI == EPI_DTANH) {
    // the WJ waves of a feature slice in a fixed order (deterministic); partial[slot / ni][feature]
    __syncthreads();
    for (int f = tid; f < BI; f += C::THREADS) {
      float t = epi_lds[f];
#pragma unroll
      for (int m = 1; m < C::WJ; ++m) t += epi_lds[m * BI + f];
      a.partial[(int64_t)(slot / a.ni) * (a.ni * BI) + it0 * BI + f] = t;
    }
  }
}

// ---- the first layer's weight gradient: dW (256, k_in <= 64) = grad^T x over all rows ----------------
// The Agent's first Linear (52 -> 256, ppo…:131,142) under loss.backward() (ppo…:352): grad (rows, 256)
// is the first tanh layer's pre-activation gradient, x (rows, k_in) the observations.  A block of 8 waves
// (two per SIMD, so one wave's staging runs beside the other's MFMAs) takes a contiguous range of K tiles
// (32 rows each) and accumulates the whole (256, 64) tile, wave w the features 64 (w & 3) .. + 63 and the
// columns 32 (w >> 2) .. + 31 (4 x 2 MFMA tiles); the grid's parts are summed by the caller.  The bytes
// are the operands once (HBM-bound: 1,024 + 4 k_in B per row); the six products keep it under that roof.
// (A first version with 4 waves, one per SIMD, ran no faster than hipBLASLt's split-K GEMM: 602 us at
// 2,097,152 rows, profiles/r05h_bench_kernel_stats_by_grid.csv -- each SIMD staged and computed in turn.)
//   grad: the K tile's 32 x 256 floats (32 KB contiguous) staged as ST_KROW into a KImg<256> image;
//   x:    its 32 x k_in floats (contiguous, k_in % 4 == 0) as 16-B chunks of 4 columns, in a 4 KB-per-plane
//         image of 16 LDS rows x 128 features: contraction row r sits at LDS row r & 15, feature
//         c + 64 (r >> 4), the 16-B chunks XOR-swizzled by kswz(row) as in KImg -- so the transposed
//         fragment reads are those of KImg (16 distinct 16-B slots per 32-lane half).  Columns k_in .. 63
//         stay zero (written once).
constexpr int FW_THREADS = 512, FW_N = 256, FW_KMAX = 64;
constexpr int FW_XPS = 16 * 256;                         // x image bytes per plane
constexpr int FW_GPS = KImg<FW_N>::PS;                   // grad image bytes per plane
constexpr int FW_BUF = 3 * FW_GPS + 3 * FW_XPS;          // 60 KB
constexpr int FW_NX = (32 * FW_KMAX / 4 + FW_THREADS - 1) / FW_THREADS;  // x chunks per thread (1)
constexpr int FW_NG = 32 * FW_N / 8 / FW_THREADS;         // grad (row, 8-feature group) pairs per thread (2)

// byte offset in one x plane of contraction row r, feature column c (c % 4 == 0): the 8-B piece of c .. c + 3
__device__ __forceinline__ int fw_xoff(int r, int c) {
  const int rho = r & 15, phi = c + 64 * (r >> 4);
  return rho * 256 + 16 * ((phi >> 3) ^ kswz(rho)) + 8 * ((phi >> 2) & 1);
}

__global__ __launch_bounds__(FW_THREADS, 1) void first_wgrad_kernel(int64_t kpairs, int32_t k_in, const float* __restrict__ grad,
                                                                      const float* __restrict__ x, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) char lds[2 * FW_BUF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x, b = blockIdx.x;
  // this block's K tiles: parts differ by at most one K-tile pair
  const int64_t kt0 = 2 * ((int64_t)b * kpairs / G), kn = 2 * (((int64_t)b + 1) * kpairs / G) - kt0;
  const int xchunks = 8 * k_in;  // 16-B chunks of one K tile of x
  // zero both x images once: the columns k_in .. 63 are never written
  for (int i = tid; i < 2 * 3 * FW_XPS / 16; i += FW_THREADS) {
    const int buf = i / (3 * FW_XPS / 16), o = i % (3 * FW_XPS / 16);
    *reinterpret_cast<u32x4*>(lds + buf * FW_BUF + 3 * FW_GPS + 16 * o) = (u32x4){0u, 0u, 0u, 0u};
  }
  struct St {
    u32x4 g[FW_NG][2];
    u32x4 x[FW_NX];
  };
  int64_t f_kt = 0;
  auto gload = [&](St& s) {
    const int64_t kt = kt0 + (f_kt < kn ? f_kt : kn - 1);  // past the last: re-load it (in bounds, unused)
    ++f_kt;
    const float* gsrc = grad + kt * 32 * FW_N;
#pragma unroll
    for (int u = 0; u < FW_NG; ++u) {
      const int pr = tid + FW_THREADS * u, row = pr >> 5, cc = pr & 31;  // 8 consecutive features of one row
      s.g[u][0] = *reinterpret_cast<const u32x4*>(gsrc + row * FW_N + 8 * cc);
      s.g[u][1] = *reinterpret_cast<const u32x4*>(gsrc + row * FW_N + 8 * cc + 4);
    }
    const float* xsrc = x + kt * 32 * k_in;
#pragma unroll
    for (int u = 0; u < FW_NX; ++u) {
      const int ch = tid + FW_THREADS * u;
      if (ch < xchunks) s.x[u] = *reinterpret_cast<const u32x4*>(xsrc + 4 * ch);
    }
  };
  auto swrite = [&](const St& s, int buf) {
    char* gimg = lds + buf * FW_BUF;
#pragma unroll
    for (int u = 0; u < FW_NG; ++u) {
      const int pr = tid + FW_THREADS * u, row = pr >> 5, cc = pr & 31;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = __uint_as_float(s.g[u][e >> 2][e & 3]);
      u32x4 hi, mid, lo;
      split8(v, hi, mid, lo);
      char* d = gimg + (cc >> 4) * KImg<FW_N>::SUB + row * 256 + 16 * ((cc & 15) ^ kswz(row));
      *reinterpret_cast<u32x4*>(d) = hi;
      *reinterpret_cast<u32x4*>(d + FW_GPS) = mid;
      *reinterpret_cast<u32x4*>(d + 2 * FW_GPS) = lo;
    }
    char* ximg = lds + buf * FW_BUF + 3 * FW_GPS;
    const int cpr = k_in >> 2;  // chunks per row
#pragma unroll
    for (int u = 0; u < FW_NX; ++u) {
      const int ch = tid + FW_THREADS * u;
      if (ch < xchunks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = __uint_as_float(s.x[u][e]);
          v[4 + e] = 0.f;
        }
        u32x4 hi, mid, lo;
        split8(v, hi, mid, lo);
        char* d = ximg + fw_xoff(ch / cpr, 4 * (ch % cpr));
        *reinterpret_cast<uint2*>(d) = (uint2){hi[0], hi[1]};
        *reinterpret_cast<uint2*>(d + FW_XPS) = (uint2){mid[0], mid[1]};
        *reinterpret_cast<uint2*>(d + 2 * FW_XPS) = (uint2){lo[0], lo[1]};
      }
    }
  };
  const int fs = wv & 3, cs = wv >> 2;  // the wave's 64-feature slice and 32-column half
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int q = (lane >> 2) & 3, p = lane & 3, fg = lane >> 4;
  auto mfma_tile = [&](int buf) {
    const char* gk = lds + buf * FW_BUF;
    const char* xk = lds + buf * FW_BUF + 3 * FW_GPS;
    u32x4 pf[3][4], qf[3][2];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int i0 = 64 * fs + 16 * i;
        pf[pl][i] = tr_frag(gk + pl * FW_GPS + kfrag_off(i0, lane, 0), gk + pl * FW_GPS + kfrag_off(i0, lane, 1));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // contraction rows 8 fg + 4 h + q, columns 16 (2 cs + j) + 4 p .. + 3
        const int r0 = 8 * fg + q, c0 = 16 * (2 * cs + j) + 4 * p;
        qf[pl][j] = tr_frag(xk + pl * FW_XPS + fw_xoff(r0, c0), xk + pl * FW_XPS + fw_xoff(r0 + 4, c0));
      }
    }
    constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
    constexpr int QP[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
    for (int xx = 0; xx < 6; ++xx)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pf[PP[xx]][i]),
                                                              __builtin_bit_cast(bf16x8, qf[QP[xx]][j]), acc[i][j], 0, 0, 0);
  };
  St r0, r1;
  __syncthreads();  // the zeroed x images before any staging write lands beside them
  gload(r0);
  swrite(r0, 0);
  gload(r1);
  gload(r0);
  __syncthreads();
  for (int64_t kt = 0; kt < kn; kt += 2) {
    mfma_tile(0);
    swrite(r1, 1);
    __syncthreads();
    gload(r1);
    mfma_tile(1);
    swrite(r0, 0);
    __syncthreads();
    gload(r0);
  }
  // lane holds D[f = 64 fs + 16 i + 4 fg + r][c = 16 (2 cs + j) + fr]; columns past k_in are zero and not stored
  const int fr = lane & 15;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = 16 * (2 * cs + j) + fr;
    if (c < k_in) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) partial[((int64_t)b * FW_N + 64 * fs + 16 * i + 4 * fg + r) * k_in + c] = acc[i][j][r];
    }
  }
}

// parts: enough K-tile pairs per block to amortise its epilogue (>= 8 pairs), at most one block per CU
static int fw_parts(int64_t rows) {
  const int64_t pairs = rows / (2 * KT);
  int64_t g = pairs / 8;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  return (int)g;
}

constexpr int kGridCus = 256;  // persistent grid sized for MI355X on every device (fixed partial layout)

struct Plan {
  int32_t ni, nj, splits, items, grid;
  int64_t kpairs;
};

// forward / backward: exact shapes only (the update's minibatches): rows % BJ, n % BI, k % 64
template <class C>
static bool fb_shape_ok(int64_t rows, int32_t k, int32_t n) {
  return rows > 0 && rows % C::BJ == 0 && rows / C::BJ <= (1 << 22) && n > 0 && n % C::BI == 0 && n <= 4096 &&
         k > 0 && k % (2 * KT) == 0 && k <= 65536 && (rows / C::BJ) * (n / C::BI) <= 0x3fffffff;
}

template <class C>
static Plan fb_plan(int64_t rows, int32_t k, int32_t n) {
  Plan p;
  p.ni = n / C::BI;
  p.nj = (int32_t)(rows / C::BJ);
  p.kpairs = k / (2 * KT);
  p.splits = 1;
  p.items = p.ni * p.nj;
  int g = kGridCus * C::BPC;
  g -= g % (8 * p.ni);  // a fixed i tile per block, 8 XCD slots
  p.grid = (g > 0 && g < p.items) ? g : p.items;
  return p;
}

// the forward / backward block for n features: CfgB where n % 256 == 0, else CfgA (n % 128); the
// host functions below take the chosen configuration as their first argument
template <class F>
static auto with_fb_cfg(int32_t n, F&& f) {
  return n > 0 && n % CfgB::BI == 0 ? f(CfgB{}) : f(CfgA{});
}

// weight gradient: dW (n_out, k_in) = grad^T x over `rows`: k_in % 128, n_out % 256, rows % 64;
// S contraction parts so that the ni * nj * S items fill the persistent grid (S <= the K-tile pairs;
// the parts differ by at most one pair: any row count that is a multiple of 64 fills the grid)
static bool wg_shape_ok(int64_t rows, int32_t n_out, int32_t k_in) {
  return rows > 0 && rows % (2 * KT) == 0 && rows <= (int64_t(1) << 36) && k_in > 0 && k_in % CfgA::BI == 0 &&
         k_in <= 4096 && n_out > 0 && n_out % CfgA::BJ == 0 && n_out <= 4096;
}

static Plan wg_plan(int64_t rows, int32_t n_out, int32_t k_in) {
  Plan p;
  p.ni = k_in / CfgA::BI;
  p.nj = n_out / CfgA::BJ;
  const int64_t pairs = rows / (2 * KT);  // K-tile pairs
  const int tiles = p.ni * p.nj;
  int64_t s = kGridCus * CfgA::BPC / tiles;
  if (s < 1) s = 1;
  if (s > pairs) s = pairs;
  p.splits = (int32_t)s;
  p.kpairs = pairs;
  p.items = tiles * s;
  p.grid = p.items < kGridCus * CfgA::BPC ? p.items : kGridCus * CfgA::BPC;
  p.grid -= (p.grid % 8 && p.grid > 8) ? p.grid % 8 : 0;
  return p;
}

template <int EPI, int SP, int SQ, class C, int KO = 0>
static int launch(void* stream, Args a, const Plan& pl) {
  a.ni = pl.ni;
  a.nj = pl.nj;
  a.kpairs = pl.kpairs;
  a.items = pl.items;
  a.splits = pl.splits;
  hipLaunchKernelGGL((gemm_x6_kernel<EPI, SP, SQ, C, KO>), dim3((unsigned)pl.grid), dim3(C::THREADS), 0,
                     (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

static bool misaligned(const void* p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) != 0; }

// the weight operand's planes: w (n, k) fp32 -> w_split, the tile-ordered LDS images of its bf16
// planes (3 n k uint16, split_image_kernel), which the GEMM copies with global_load_lds
template <class C>
static int split_weight(void* stream, const float* w, int64_t n, int64_t k, uint16_t* w_split) {
  const int64_t units = n * k / 8;
  hipLaunchKernelGGL(split_image_kernel<C::BI>, dim3((unsigned)((units + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, w, n, k, w_split);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

// forward / backward arguments: P = the weight's planes, Q = the activations (K-contiguous)
static Args fb_args(int32_t k, int32_t n, const uint16_t* w_split, const float* q, float* out) {
  Args a{};
  a.ldp = k;
  a.ldq = k;
  a.p = w_split;
  a.q = q;
  a.ldo = n;
  a.out = out;
  return a;
}

// ---- the first hidden layer's forward on the bf16 matrix cores: y = tanh(x W^T + b) ---------------------
// The Agent's first Linear + Tanh (nn.Linear(52, 256), ppo…:131,142) over the update's minibatch and the
// rollout's observations.  On the fp32 MFMA (vss_update.hip first_layer_kernel) its 56 GFLOP at 2,097,152
// rows cost 0.46 ms of matrix time before the tanh and the 2.1 GB of stores.  Here each of 8 waves per
// block takes 16-row slabs on its own: x straight from global memory (lane = row fr, k group fg: two 16-B
// loads per K step of 32, k >= k_in zero), split into hi / mid / lo in registers (split8); W's three
// planes were split once per block into LDS as the A fragments ([ks][plane][i tile][fg][fr] x 16 B,
// 96 KB: a fragment read is 16 consecutive 16-B slots per 16-lane group); per slab 16 i tiles x 2 K
// steps x 6 products (the x6 order, smallest first), then bias + tanh and 16-B stores of 4 consecutive
// features of a row.  No barrier after the W split, so one wave's tanh and stores run beside the other
// waves' MFMAs.  The x6 error bound applies (products exact, the dropped terms < 2^-23 |a||b|).
constexpr int FL_WAVES = 8, FL_THREADS = 64 * FL_WAVES;
// Measured at 2,097,152 rows (profiles/r05_first_layer_x6.log): 650-670 us against the fp32-MFMA kernel's
// 830-870 us; without the stores (timing only) 419 us, without the tanh 648 us -- the HBM stores set it.
// Not kept, all slower or equal: 16 waves x 128-feature halves (810 us), nontemporal stores (734 us),
// the stores as whole 128-B lines through a per-wave LDS transpose (653 us), and a branch-free
// software pipeline that interleaves one slab's tanh / stores with the next slab's MFMAs in every wave
// (two accumulator sets, buffer-descriptor stores; 670-701 us).
__global__ __launch_bounds__(FL_THREADS) void first_layer_x6_kernel(int64_t rows, int k, const float* __restrict__ x,
                                                                    const float* __restrict__ w,
                                                                    const float* __restrict__ bias,
                                                                    float* __restrict__ y) {
  __shared__ u32x4 wimg[2 * 3 * 16 * 64];  // [ks][plane][i tile][fg * 16 + fr]
  __shared__ float bl[256];
  for (int p = threadIdx.x; p < 256 * 8; p += FL_THREADS) {  // (feature, k group of 8) pairs
    const int f = p >> 3, g = p & 7;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = 8 * g + e;
      v[e] = kk < k ? w[(int64_t)f * k + kk] : 0.0f;
    }
    u32x4 pl[3];
    split8(v, pl[0], pl[1], pl[2]);
    const int ks = g >> 2, fg = g & 3, it = f >> 4, fr = f & 15;
#pragma unroll
    for (int q = 0; q < 3; ++q) wimg[((ks * 3 + q) * 16 + it) * 64 + fg * 16 + fr] = pl[q];
  }
  for (int i = threadIdx.x; i < 256; i += FL_THREADS) bl[i] = bias[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
  const int64_t slabs = (rows + 15) / 16, step = (int64_t)gridDim.x * FL_WAVES;
  auto load_x = [&](int64_t sl, float4 (&xr)[2][2]) __attribute__((always_inline)) {
    const int64_t row = sl * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k0 = 32 * ks + 8 * fg + 4 * h;
        xr[ks][h] = (row < rows && k0 + 4 <= k) ? *reinterpret_cast<const float4*>(x + row * k + k0)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  };
  // the six products, smallest first (gemm_x6_kernel's order): lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
  constexpr int PP[6] = {2, 0, 1, 1, 0, 0};
  constexpr int QP[6] = {0, 2, 1, 0, 1, 0};
  int64_t sl = (int64_t)blockIdx.x * FL_WAVES + wv;
  float4 xr[2][2];
  if (sl < slabs) load_x(sl, xr);
  for (; sl < slabs; sl += step) {
    u32x4 xp[2][3];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float v[8] = {xr[ks][0].x, xr[ks][0].y, xr[ks][0].z, xr[ks][0].w,
                          xr[ks][1].x, xr[ks][1].y, xr[ks][1].z, xr[ks][1].w};
      split8(v, xp[ks][0], xp[ks][1], xp[ks][2]);
    }
    if (sl + step < slabs) load_x(sl + step, xr);  // the next slab's x lands during this one
    f32x4 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // 8 steps (group of 4 i tiles, K step); one step's 12 fragments live at a time (without the fences
    // the compiler hoists all 96 fragment reads of the slab, 384 VGPRs, and spills)
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const int ig = st >> 1, ks = st & 1;
      u32x4 pf[3][4];
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) pf[q][ii] = wimg[((ks * 3 + q) * 16 + 4 * ig + ii) * 64 + lane];
#pragma unroll
      for (int xx = 0; xx < 6; ++xx)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
          acc[4 * ig + ii] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pf[PP[xx]][ii]),
                                                                     __builtin_bit_cast(bf16x8, xp[ks][QP[xx]]),
                                                                     acc[4 * ig + ii], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int64_t row = sl * 16 + fr;
    if (row < rows) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int f0 = 16 * i + 4 * fg;
        f32x4 v = acc[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tanh_f32(v[r] + bl[f0 + r]);
        *reinterpret_cast<f32x4*>(y + row * 256 + f0) = v;
      }
    }
  }
}

}  // namespace vx6

extern "C" {

int vss_linear_tanh_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                           const float* bias, float* y, uint16_t* w_split) {
  using namespace vx6;
  return with_fb_cfg(n_out, [&](auto cfg) {
    using C = decltype(cfg);
    if (!fb_shape_ok<C>(rows, k_in, n_out) || (w && misaligned(w)) || misaligned(x) || misaligned(y) || !bias ||
        misaligned(w_split))
      return (int)VSS_E_ARG;
    int rc = w ? split_weight<C>(stream, w, n_out, k_in, w_split) : VSS_OK;
    if (rc != VSS_OK) return rc;
    Args a = fb_args(k_in, n_out, w_split, x, y);
    a.bias = bias;
    return launch<EPI_TANH, ST_DMA, ST_ROW, C>(stream, a, fb_plan<C>(rows, k_in, n_out));
  });
}

int vss_linear_tanh_out_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                               const float* bias, float* y, int32_t k_out, const float* w_out, float* out_part,
                               uint16_t* w_split) {
  using namespace vx6;
  return with_fb_cfg(n_out, [&](auto cfg) {
    using C = decltype(cfg);
    if (!fb_shape_ok<C>(rows, k_in, n_out) || n_out != 256 || misaligned(x) || (w && misaligned(w)) || misaligned(y) ||
        !bias || !w_out || !out_part || !(k_out == 1 || k_out == 2 || k_out == 6) || misaligned(w_split))
      return (int)VSS_E_ARG;
    int rc = w ? split_weight<C>(stream, w, n_out, k_in, w_split) : VSS_OK;
    if (rc != VSS_OK) return rc;
    Args a = fb_args(k_in, n_out, w_split, x, y);
    a.bias = bias;
    a.w_out = w_out;
    a.out_part = out_part;
    const Plan pl = fb_plan<C>(rows, k_in, n_out);
    if (k_out == 1) return launch<EPI_TANH_OUT, ST_DMA, ST_ROW, C, 1>(stream, a, pl);
    if (k_out == 2) return launch<EPI_TANH_OUT, ST_DMA, ST_ROW, C, 2>(stream, a, pl);
    return launch<EPI_TANH_OUT, ST_DMA, ST_ROW, C, 6>(stream, a, pl);
  });
}

int64_t vss_linear_tanh_loss_blocks_bf16x6(int64_t rows, int32_t k_in, int32_t n_out) {
  using namespace vx6;
  if (n_out != 256 || !fb_shape_ok<CfgB>(rows, k_in, n_out)) return -1;
  return fb_plan<CfgB>(rows, k_in, n_out).grid;
}

int vss_linear_tanh_loss_bf16x6(void* stream, int32_t role, int64_t rows_pad, int64_t rows, int32_t k_in, int32_t n_out,
                                const float* x, const float* bias, int32_t k_out, const float* w_out, const float* b_out,
                                const float* action, const float* logprob_old, const float* adv, const double* adv_part,
                                int32_t adv_nparts, double adv_count, const float* logstd, const float* returns,
                                const float* values_old, float clip_coef, float clip_lo, float clip_hi, float vf_coef,
                                int32_t clip_vloss, float* grad_in, float* part_cs, float* part_dwo, float* part_stats,
                                const uint16_t* w_split) {
  using namespace vx6;
  using C = CfgB;
  const bool actor = role == 0;
  if ((role != 0 && role != 1) || n_out != 256 || !fb_shape_ok<C>(rows_pad, k_in, n_out) || rows <= 0 || rows > rows_pad ||
      misaligned(x) || misaligned(grad_in) || misaligned(w_split) || !bias || !w_out || !b_out || !part_cs || !part_dwo ||
      !part_stats || (actor && (k_out < 1 || k_out > 2 || !action || !logprob_old || !adv || !logstd ||
                                (adv_part && (adv_nparts < 1 || !(adv_count > 1.0))))) ||
      (!actor && (k_out != 1 || !returns || (clip_vloss && !values_old))))
    return VSS_E_ARG;
  Args a = fb_args(k_in, n_out, w_split, x, grad_in);
  a.bias = bias;
  a.w_out = w_out;
  a.b_out = b_out;
  a.l_act = action;
  a.l_logp = logprob_old;
  a.l_adv = adv;
  a.adv_part = adv_part;
  a.adv_nparts = adv_nparts;
  a.adv_count = adv_count;
  a.logstd = logstd;
  a.l_ret = returns;
  a.l_val = values_old;
  a.clip = clip_coef;
  a.clip_lo = clip_lo;
  a.clip_hi = clip_hi;
  a.vf_coef = vf_coef;
  a.inv_n = 1.0f / (float)rows;
  a.clip_vloss = clip_vloss;
  a.rows_real = rows;
  a.part_cs = part_cs;
  a.part_dwo = part_dwo;
  a.part_stats = part_stats;
  const Plan pl = fb_plan<C>(rows_pad, k_in, n_out);
  if (!actor) return launch<EPI_LOSS_C, ST_DMA, ST_ROW, C, 1>(stream, a, pl);
  if (k_out == 1) return launch<EPI_LOSS_A, ST_DMA, ST_ROW, C, 1>(stream, a, pl);
  return launch<EPI_LOSS_A, ST_DMA, ST_ROW, C, 2>(stream, a, pl);
}

int64_t vss_linear_tanh_backward_chunks_bf16x6(int64_t rows, int32_t k_next, int32_t n_out) {
  using namespace vx6;
  return with_fb_cfg(n_out, [&](auto cfg) -> int64_t {
    using C = decltype(cfg);
    if (!fb_shape_ok<C>(rows, k_next, n_out)) return -1;
    const Plan pl = fb_plan<C>(rows, k_next, n_out);
    return pl.grid / pl.ni;
  });
}

int vss_linear_tanh_backward_bf16x6(void* stream, int64_t rows, int32_t k_next, int32_t n_out, const float* grad_next,
                                    const float* w_next_t, const float* y, float* grad_in, float* bias_partial,
                                    uint16_t* w_split) {
  using namespace vx6;
  return with_fb_cfg(n_out, [&](auto cfg) {
    using C = decltype(cfg);
    if (!fb_shape_ok<C>(rows, k_next, n_out) || misaligned(grad_next) || (w_next_t && misaligned(w_next_t)) ||
        misaligned(y) || misaligned(grad_in) || misaligned(bias_partial) || misaligned(w_split))
      return (int)VSS_E_ARG;
    int rc = w_next_t ? split_weight<C>(stream, w_next_t, n_out, k_next, w_split) : VSS_OK;
    if (rc != VSS_OK) return rc;
    Args a = fb_args(k_next, n_out, w_split, grad_next, grad_in);
    a.y = y;
    a.partial = bias_partial;
    return launch<EPI_DTANH, ST_DMA, ST_ROW, C>(stream, a, fb_plan<C>(rows, k_next, n_out));
  });
}

int vss_weight_planes_bf16x6(void* stream, int32_t count, const float* const* w, const int32_t* n, const int32_t* k,
                             const int32_t* transpose, uint16_t* const* w_split) {
  using namespace vx6;
  if (count < 1 || count > kMaxPlaneJobs || !w || !n || !k || !transpose || !w_split) return VSS_E_ARG;
  PlaneJobs jobs{};
  int64_t blocks = 0;
  for (int q = 0; q < count; ++q) {
    const int32_t nq = n[q], kq = k[q];
    // the image's row tile is the forward / backward block's (with_fb_cfg): 256 where n % 256 == 0
    if (nq <= 0 || nq % CfgA::BI || nq > 4096 || kq <= 0 || kq % (2 * KT) || kq > 65536 || !w[q] ||
        misaligned(w_split[q]) || (transpose[q] != 0 && transpose[q] != 1) ||
        (!transpose[q] && misaligned(w[q])))
      return VSS_E_ARG;
    jobs.j[q] = PlaneJob{w[q], w_split[q], nq, kq, transpose[q], nq % CfgB::BI == 0 ? CfgB::BI : CfgA::BI};
    const int64_t b = ((int64_t)nq * kq / 8 + 255) / 256;
    if (b > blocks) blocks = b;
  }
  hipLaunchKernelGGL(plane_images_kernel, dim3((unsigned)blocks, (unsigned)count), dim3(256), 0, (hipStream_t)stream,
                     jobs);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int64_t vss_weight_grad_chunks_bf16x6(int64_t rows, int32_t n_out, int32_t k_in) {
  using namespace vx6;
  if (!wg_shape_ok(rows, n_out, k_in)) return -1;
  return wg_plan(rows, n_out, k_in).splits;
}

int vss_weight_grad_bf16x6(void* stream, int64_t rows, int32_t n_out, int32_t k_in, const float* grad, const float* x,
                           float* partial) {
  using namespace vx6;
  if (!wg_shape_ok(rows, n_out, k_in) || misaligned(grad) || misaligned(x) || misaligned(partial)) return VSS_E_ARG;
  Args a{};
  a.ldp = k_in;
  a.ldq = n_out;
  a.p = x;
  a.q = grad;
  a.ldo = k_in;
  a.out = partial;
  return launch<EPI_WGRAD, ST_KROW, ST_KROW, CfgA>(stream, a, wg_plan(rows, n_out, k_in));
}

int64_t vss_first_weight_grad_chunks_bf16x6(int64_t rows, int32_t n_out, int32_t k_in) {
  using namespace vx6;
  if (rows <= 0 || rows % (2 * KT) || rows > (int64_t(1) << 36) || n_out != FW_N || k_in <= 0 || k_in > FW_KMAX ||
      k_in % 4)
    return -1;
  return fw_parts(rows);
}

int vss_first_weight_grad_bf16x6(void* stream, int64_t rows, int32_t n_out, int32_t k_in, const float* grad,
                                 const float* x, float* partial) {
  using namespace vx6;
  if (vss_first_weight_grad_chunks_bf16x6(rows, n_out, k_in) < 0 || misaligned(grad) || misaligned(x) || !partial)
    return VSS_E_ARG;
  const int g = fw_parts(rows);
  hipLaunchKernelGGL(first_wgrad_kernel, dim3((unsigned)g), dim3(FW_THREADS), 0, (hipStream_t)stream,
                     (int64_t)(rows / (2 * KT)), k_in, grad, x, partial);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

int vss_first_layer_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                           const float* bias, float* y) {
  using namespace vx6;
  if (rows < 0 || n_out != 256 || k_in <= 0 || k_in > 64 || k_in % 4 != 0 || misaligned(x) || !w || !bias ||
      misaligned(y))
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  int64_t g = ((rows + 15) / 16 + FL_WAVES - 1) / FL_WAVES;
  if (g > 256) g = 256;  // one block per CU (96 KB of W planes), persistent over the slabs
  hipLaunchKernelGGL(first_layer_x6_kernel, dim3((unsigned)g), dim3(FL_THREADS), 0, (hipStream_t)stream, rows, k_in, x,
                     w, bias, y);
  return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH;
}

}  // extern "C"
