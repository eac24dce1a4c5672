// vss_step.hip — MI355X (gfx950) kernels behind the C ABI of include/vss.h.
//
// One VSS field (a 3v3 match) per lane, 64 fields per wave / workgroup.  Per step a lane
//   1. loads its field's 46 live fp32 state channels from the SoA state (coalesced, 256 B per
//      wave-instruction per channel) plus progress/reset/rng counter,
//   2. gathers its 12 actions (and, in SA/CMA/DMA mode, the OU action buffer) through an LDS
//      transpose (16-B coalesced global loads of the wave's contiguous AoS block),
//   3. runs the 2D physics for NSUB substeps in registers,
//   4. computes rewards / dones (envs/vss.py:218-265, 578-655),
//   5. writes the terminal observation, resets done fields (Philox rejection sampling,
//      envs/vss.py:267-333), writes the observation — both observations through an LDS
//      record (58 floats per field) that the wave streams out with 16-B coalesced stores in
//      the (N, A, 52) layout, using a compile-time gather table (envs/vss.py:530-575),
//   6. stores state, bookkeeping and the AoS reward block (LDS transpose again).
// Everything is float32 with FMA contraction disabled (-ffp-contract=off and the pragma
// below): results are bit-identical to the CPU oracle (oracle/vss_oracle.c).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "../../include/vss.h"

#pragma clang fp contract(off)

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vss_step.hip targets gfx950 (CDNA4) only: wait_loads() and v_permlane32_swap are gfx950 encodings"
#endif

namespace vss {

constexpr int kWave = 64;
// Fields per step/rollout wave (one wave per workgroup; all 64 lanes take part in the streams).
// 32, not 64: at 65,536 fields that is 2,048 waves = 2 per SIMD, so one wave's physics overlaps the
// other wave's stores, and lanes L and L + 32 share a field, splitting its per-robot physics
// (physics_split).  Measured (profiles/r01_ablate_*): FULL 48.8 -> 42.7 us with 32 fields per wave,
// -> 40.8 us with the split; SA 27.2 -> 25.9 us.  16 and 24 are slower (profiles/r02_ablate_fields_
// per_wave_*: LDS and VGPRs allow fewer than 3 waves per SIMD).  A persistent variant (1,024 waves x
// 2 batches, next batch prefetched) was 12-33 % slower (profiles/r02_ablate_persist_*.log).
constexpr int kFpw = 32;
constexpr int kRec = 59;  // LDS floats per field record (58 used, odd stride: no bank conflicts)

// ---- model constants (reference values cited in oracle/vss_oracle.c) --------
constexpr int NSUB = 2;  // Isaac Gym's default substeps per control step
#define K_H 0.025f
#define K_HH 0.0125f
#define K_FIELD_HX 0.75f
#define K_FIELD_HY 0.65f
#define K_GOAL_HY 0.2f
#define K_GOAL_BACK_X 0.85f
#define K_BALL_R 0.02134f
#define K_BALL_R2 0.00045539559f
#define K_ROBOT_HALF 0.035f
#define K_ROBOT_R 0.04f
#define K_RR_DIST 0.08f
#define K_RR_DIST2 0.0064f
#define K_WHEEL_RAD_S 42.0f
#define K_WHEEL_R 0.024f
#define K_HALF_TRACK 0.03375f
#define K_INV_TRACK 14.814815f
#define K_DV 0.15f
#define K_DL 0.171675f
#define K_BALL_DAMP 0.99625f
#define K_W_ROBOT_BR 0.09465021f
#define K_W_BALL_BR 0.90534979f
#define K_MIN_DIST 0.07f
#define K_TWO_PI 6.2831855f
#define K_PI 3.1415927f
#define K_OU_THETA 0.1f
#define K_OU_SIGMA 0.15f
constexpr int kMaxRejectRounds = 64;
constexpr uint32_t kPurposeOU = 1u, kPurposePos = 2u, kPurposeAng = 3u, kExternal = 0x80u;

// ---- observation gather table ---------------------------------------------------------------
// For float4 index j4 (0..77) of a field's (6, 52) observation block: 4 bytes, each
// (source index into the 58-float LDS record) | 0x80 if the value is negated (yellow mirror).
// Observation records in LDS.  Plain record (kRec = 59 floats): ball (4) + 6 x (x, y, vx, vy, cos,
// sin, w, aL, aR).  The FULL contract (A = 6 agents) appends the 40 slots that the yellow view
// negates (ball 4 + 6 x (x, y, vx, vy, cos, sin)), already negated: the streams then gather plain
// copies only.  Record stride kRecObs6 = 99 floats (odd: conflict-free per-lane writes).
constexpr int kRecObs6 = kRec + 40;
template <int A>
constexpr int obs_rec() { return A == 6 ? kRecObs6 : kRec; }
constexpr int mirror_slot(int src) { return src < 4 ? kRec + src : kRec + 4 + ((src - 4) / 9) * 6 + (src - 4) % 9; }

// Gather table for the (2,3,52) per-field observation block, one entry per float4: two words,
// each two 16-bit LDS byte offsets within the field's record (source slot x 4; yellow-view
// negated values point into the mirror slots).  A < 6 contracts use the first 13 x A entries
// (blue agents: no mirror slots), so one table serves every record stride.
struct ObsTable {
  uint32_t w[2 * 78];
};

constexpr ObsTable make_obs_table() {
  ObsTable t{};
  for (int j = 0; j < 312; ++j) {
    int a = j / 52, e = j % 52, team = a / 3, idx = a % 3;
    int src = 0;
    bool neg = false;
    if (e < 4) {
      src = e;
      neg = team == 1;
    } else if (e < 31) {
      int k = (e - 4) / 9, q = (e - 4) % 9;
      int r = team * 3 + (idx + k) % 3;
      src = 4 + r * 9 + q;
      neg = team == 1 && q < 6;
    } else {
      int k = (e - 31) / 7, q = (e - 31) % 7;
      int r = (1 - team) * 3 + k;
      src = 4 + r * 9 + q;
      neg = team == 1 && q < 6;
    }
    uint32_t off = 4u * (uint32_t)(neg ? mirror_slot(src) : src);
    t.w[j / 2] |= off << (16 * (j % 2));
  }
  return t;
}

__constant__ ObsTable kObsTab = make_obs_table();
constexpr int kTabWords = 2 * 78;

// The gather table is copied into LDS once per wave, at the start (before any store): a lane-
// indexed read of the __constant__ table is a global_load, and on gfx9 vmcnt counts stores too, so
// waiting for a table load issued between the stream's stores drains every store before it
// (measured in the ISA: an s_waitcnt vmcnt(0) per unrolled stream iteration).  ds_read waits
// on lgkmcnt instead, which the stores do not touch.
__device__ __forceinline__ void stage_obs_table(uint32_t* tab, int lane) {
  for (int i = lane; i < kTabWords; i += kWave) tab[i] = kObsTab.w[i];
}

// ---- math (transcendental-free; identical op sequence in oracle/vss_oracle.c) ----------------
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

__device__ __forceinline__ void philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2,
                                       uint32_t c3, uint32_t out[4]) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one 32 x 32 -> 64-bit product each (v_mad_u64_u32) instead of separate mul_hi / mul_lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 5.9604645e-08f; }
__device__ __forceinline__ float u01_open0(uint32_t x) { return (float)((x >> 8) + 1u) * 5.9604645e-08f; }

__device__ __forceinline__ void sincos_poly(float r, float& s, float& c) {
  float r2 = r * r;
  s = r + r * r2 * (-0.16666667f + r2 * (0.008333334f + r2 * (-1.9841270e-4f + r2 * 2.7557319e-6f)));
  c = 1.0f + r2 * (-0.5f + r2 * (0.041666668f + r2 * (-1.3888889e-3f + r2 * (2.4801587e-5f + r2 * (-2.7557319e-7f)))));
}

__device__ __forceinline__ void sincos_small(float x, float& s, float& c) {
  if (fabsf(x) < 0.78f) {  // |x| < pi/4: no reduction (always the case for yaw steps)
    sincos_poly(x, s, c);
    return;
  }
  int k = (int)(x * 0.63661977f + (x >= 0.0f ? 0.5f : -0.5f));
  float kf = (float)k;
  float r = (x - kf * 1.5707964f) - kf * (-4.3711390e-8f);
  float sr, cr;
  sincos_poly(r, sr, cr);
  if (k == 0) { s = sr; c = cr; }
  else if (k == 1) { s = cr; c = -sr; }
  else if (k == -1) { s = -cr; c = sr; }
  else { s = -sr; c = -cr; }
}

__device__ __forceinline__ void sincos_turn(float u, float& s, float& c) {
  float v = u * 4.0f;
  int q = (int)v;
  float t = v - (float)q;
  float r = (t - 0.5f) * 1.5707964f;
  float sr, cr;
  sincos_poly(r, sr, cr);
  float cp = (cr - sr) * 0.70710677f;
  float sp = (cr + sr) * 0.70710677f;
  if (q == 0) { c = cp; s = sp; }
  else if (q == 1) { c = -sp; s = cp; }
  else if (q == 2) { c = -cp; s = -sp; }
  else { c = sp; s = -cp; }
}

__device__ __forceinline__ float logf_poly(float x) {
  uint32_t u = __float_as_uint(x);
  int e = (int)((u >> 23) & 0xffu) - 127;
  float m = __uint_as_float((u & 0x7fffffu) | 0x3f800000u);
  if (m > 1.4142135f) { m = m * 0.5f; e = e + 1; }
  float s = (m - 1.0f) / (m + 1.0f);
  float s2 = s * s;
  float p = 2.0f + s2 * (0.6666667f + s2 * (0.4f + s2 * (0.2857143f + s2 * (0.22222222f + s2 * 0.18181819f))));
  return (float)e * 0.69314718f + s * p;
}


// ---- per-field body state in registers ---------------------------------------------------------
struct Bodies {
  float bx, by, bvx, bvy;
  float x[6], y[6], qz[6], qw[6], vx[6], vy[6], w[6];
  float c[6], s[6];
};

__device__ __forceinline__ void heading(Bodies& b, int i) {
  b.c[i] = b.qw[i] * b.qw[i] - b.qz[i] * b.qz[i];
  b.s[i] = 2.0f * b.qw[i] * b.qz[i];
}

__device__ __forceinline__ void contact_robot_robot(Bodies& b, int i, int j) {
  float dx = b.x[j] - b.x[i], dy = b.y[j] - b.y[i];
  float d2 = dx * dx + dy * dy;
  if (d2 < K_RR_DIST2) {
    float d = sqrtf(d2);
    float nx = 1.0f, ny = 0.0f;
    if (d > 1e-9f) { float inv = 1.0f / d; nx = dx * inv; ny = dy * inv; }
    float half = (K_RR_DIST - d) * 0.5f;
    b.x[i] = b.x[i] - nx * half; b.y[i] = b.y[i] - ny * half;
    b.x[j] = b.x[j] + nx * half; b.y[j] = b.y[j] + ny * half;
    float vn = (b.vx[j] - b.vx[i]) * nx + (b.vy[j] - b.vy[i]) * ny;
    if (vn < 0.0f) {
      float jn = vn * 0.5f;
      b.vx[i] = b.vx[i] + nx * jn; b.vy[i] = b.vy[i] + ny * jn;
      b.vx[j] = b.vx[j] - nx * jn; b.vy[j] = b.vy[j] - ny * jn;
    }
  }
}

__device__ __forceinline__ void contact_ball_robot(Bodies& b, int i) {
  float dx = b.bx - b.x[i], dy = b.by - b.y[i];
  float c = b.c[i], s = b.s[i];
  float lx = c * dx + s * dy;
  float ly = c * dy - s * dx;
  float cx = clampf(lx, -K_ROBOT_HALF, K_ROBOT_HALF);
  float cy = clampf(ly, -K_ROBOT_HALF, K_ROBOT_HALF);
  float ex = lx - cx, ey = ly - cy;
  float d2 = ex * ex + ey * ey;
  if (d2 < K_BALL_R2) {  // contact (d2 == 0: ball centre inside the box)
    float nlx, nly, pen;
    if (d2 > 0.0f) {
      float d = sqrtf(d2);
      float inv = 1.0f / d;
      nlx = ex * inv; nly = ey * inv;
      pen = K_BALL_R - d;
    } else {
      float px = K_ROBOT_HALF - fabsf(lx), py = K_ROBOT_HALF - fabsf(ly);
      if (px < py) { nlx = lx >= 0.0f ? 1.0f : -1.0f; nly = 0.0f; pen = px + K_BALL_R; }
      else { nlx = 0.0f; nly = ly >= 0.0f ? 1.0f : -1.0f; pen = py + K_BALL_R; }
    }
    float nx = c * nlx - s * nly;
    float ny = s * nlx + c * nly;
    float pr = pen * K_W_ROBOT_BR, pb = pen * K_W_BALL_BR;
    b.x[i] = b.x[i] - nx * pr; b.y[i] = b.y[i] - ny * pr;
    b.bx = b.bx + nx * pb; b.by = b.by + ny * pb;
    float vn = (b.bvx - b.vx[i]) * nx + (b.bvy - b.vy[i]) * ny;
    if (vn < 0.0f) {
      float jr = vn * K_W_ROBOT_BR, jb = vn * K_W_BALL_BR;
      b.vx[i] = b.vx[i] + nx * jr; b.vy[i] = b.vy[i] + ny * jr;
      b.bvx = b.bvx - nx * jb; b.bvy = b.bvy - ny * jb;
    }
  }
}

// Disc of radius r against the field walls (envs/vss.py:449-518), folded into x, y >= 0.
// Face contacts are select-based (no divergent branches); only the goal-post corner, which needs
// sqrt/div, branches.  Identical results to the branchy form in oracle/vss_oracle.c.
__device__ __forceinline__ void push_face(float& a, float& va, float pen) {
  const bool hit = pen > 0.0f;
  a = hit ? a - pen : a;
  va = (hit && va > 0.0f) ? 0.0f : va;
}

__device__ __forceinline__ void contact_walls(float& x, float& y, float& vx, float& vy, float r) {
  float sx = x < 0.0f ? -1.0f : 1.0f, sy = y < 0.0f ? -1.0f : 1.0f;
  float ax = fabsf(x), ay = fabsf(y);
  float avx = vx * sx, avy = vy * sy;
  const bool in_x = ax <= K_FIELD_HX, in_y = ay <= K_GOAL_HY;
  if (in_x && in_y) {  // near the goal-post corner (0.75, 0.2)
    float dx = ax - K_FIELD_HX, dy = ay - K_GOAL_HY;
    float d2 = dx * dx + dy * dy;
    if (d2 < r * r) {
      float d = sqrtf(d2);
      float nx = -1.0f, ny = 0.0f;
      if (d > 1e-9f) { float inv = 1.0f / d; nx = dx * inv; ny = dy * inv; }
      float pen = r - d;
      ax = ax + nx * pen; ay = ay + ny * pen;
      float vn = avx * nx + avy * ny;
      if (vn < 0.0f) { avx = avx - nx * vn; avy = avy - ny * vn; }
    }
  } else {
    // end-wall face (in_x, !in_y), goal-pocket side face (!in_x, in_y), or centre inside the
    // end wall (!in_x, !in_y): shortest way out
    const float px = ax - K_FIELD_HX + r, py = ay - K_GOAL_HY + r;
    const float pen_end = ax + r - K_FIELD_HX, pen_side = ay + r - K_GOAL_HY;
    const bool use_x = in_x || (!in_y && px < py);
    const float pen = in_x ? pen_end : (in_y ? pen_side : (px < py ? px : py));
    push_face(ax, avx, use_x ? pen : -1.0f);
    push_face(ay, avy, use_x ? -1.0f : pen);
  }
  push_face(ay, avy, ay + r - K_FIELD_HY);
  push_face(ax, avx, ax + r - K_GOAL_BACK_X);
  x = ax * sx; y = ay * sy; vx = avx * sx; vy = avy * sy;
}

// One robot's traction-limited differential drive (spec §3) and its explicit integration step
// (position, yaw quaternion with one Newton renormalisation, heading).  Shared by both physics
// forms below, so every robot sees the identical operation sequence.
__device__ __forceinline__ void drive_robot(float c, float s, float& vx, float& vy, float& w, float tl, float tr) {
  float vf = c * vx + s * vy;
  float vl = c * vy - s * vx;
  float wl = vf - w * K_HALF_TRACK;
  float wr = vf + w * K_HALF_TRACK;
  wl = wl + clampf(tl - wl, -K_DV, K_DV);
  wr = wr + clampf(tr - wr, -K_DV, K_DV);
  vf = (wl + wr) * 0.5f;
  w = (wr - wl) * K_INV_TRACK;
  vl = vl - clampf(vl, -K_DL, K_DL);
  vx = c * vf - s * vl;
  vy = s * vf + c * vl;
}

__device__ __forceinline__ void integrate_robot(float& x, float& y, float vx, float vy, float w, float& qz, float& qw,
                                                float& c, float& s) {
  x = x + vx * K_H;
  y = y + vy * K_H;
  float sh, ch;
  sincos_small(w * K_HH, sh, ch);
  const float nqz = qz * ch + qw * sh;
  const float nqw = qw * ch - qz * sh;
  const float k = 1.5f - 0.5f * (nqz * nqz + nqw * nqw);  // one Newton step of 1/|q|
  qz = nqz * k;
  qw = nqw * k;
  c = qw * qw - qz * qz;
  s = 2.0f * qw * qz;
}

// Both lane halves of a wave hold the same field (lane L and L + 32).  The per-robot phases
// (drive, integration, walls) run on the half's own robots (lower half 0-2, upper half 3-5), and
// one v_permlane32_swap per value writes robot k and k + 3 back into every lane's canonical
// registers; the sequential contacts (robot-robot, ball-robot) and the ball run in both halves
// on the canonical state.  Same per-robot operations as physics(): bit-identical results with
// about 28 % fewer VALU instructions per field.
__device__ __forceinline__ void exch(float v, float& lo, float& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  lo = __uint_as_float(r[0]);  // the lower half's value, in every lane
  hi = __uint_as_float(r[1]);  // the upper half's value, in every lane
}

__device__ __forceinline__ void physics_split(Bodies& b, const float a[12]) {
  const bool up = threadIdx.x >= 32;
  // this half's robots: own state (o*) is kept across the phases that leave it unchanged
  float tl[3], tr[3], ox[3], oy[3], ovx[3], ovy[3], ow[3], oqz[3], oqw[3], oc[3], os[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float al = up ? a[2 * k + 6] : a[2 * k], ar = up ? a[2 * k + 7] : a[2 * k + 1];
    tl[k] = (al * K_WHEEL_RAD_S) * K_WHEEL_R;
    tr[k] = (ar * K_WHEEL_RAD_S) * K_WHEEL_R;
    ox[k] = up ? b.x[k + 3] : b.x[k];
    oy[k] = up ? b.y[k + 3] : b.y[k];
    ovx[k] = up ? b.vx[k + 3] : b.vx[k];
    ovy[k] = up ? b.vy[k + 3] : b.vy[k];
    ow[k] = up ? b.w[k + 3] : b.w[k];
    oqz[k] = up ? b.qz[k + 3] : b.qz[k];
    oqw[k] = up ? b.qw[k + 3] : b.qw[k];
    oc[k] = oqw[k] * oqw[k] - oqz[k] * oqz[k];
    os[k] = 2.0f * oqw[k] * oqz[k];
  }
#pragma unroll 1
  for (int sub = 0; sub < NSUB; ++sub) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      drive_robot(oc[k], os[k], ovx[k], ovy[k], ow[k], tl[k], tr[k]);
      integrate_robot(ox[k], oy[k], ovx[k], ovy[k], ow[k], oqz[k], oqw[k], oc[k], os[k]);
      exch(ox[k], b.x[k], b.x[k + 3]);
      exch(oy[k], b.y[k], b.y[k + 3]);
      exch(ovx[k], b.vx[k], b.vx[k + 3]);
      exch(ovy[k], b.vy[k], b.vy[k + 3]);
      exch(oc[k], b.c[k], b.c[k + 3]);
      exch(os[k], b.s[k], b.s[k + 3]);
    }
    b.bvx = b.bvx * K_BALL_DAMP;
    b.bvy = b.bvy * K_BALL_DAMP;
    b.bx = b.bx + b.bvx * K_H;
    b.by = b.by + b.bvy * K_H;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = i + 1; j < 6; ++j) contact_robot_robot(b, i, j);
#pragma unroll
    for (int i = 0; i < 6; ++i) contact_ball_robot(b, i);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ox[k] = up ? b.x[k + 3] : b.x[k];
      oy[k] = up ? b.y[k + 3] : b.y[k];
      ovx[k] = up ? b.vx[k + 3] : b.vx[k];
      ovy[k] = up ? b.vy[k + 3] : b.vy[k];
      contact_walls(ox[k], oy[k], ovx[k], ovy[k], K_ROBOT_R);
      exch(ox[k], b.x[k], b.x[k + 3]);
      exch(oy[k], b.y[k], b.y[k + 3]);
      exch(ovx[k], b.vx[k], b.vx[k + 3]);
      exch(ovy[k], b.vy[k], b.vy[k + 3]);
    }
    contact_walls(b.bx, b.by, b.bvx, b.bvy, K_BALL_R);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    exch(ow[k], b.w[k], b.w[k + 3]);
    exch(oqz[k], b.qz[k], b.qz[k + 3]);
    exch(oqw[k], b.qw[k], b.qw[k + 3]);
  }
}

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt untouched: 0x0F70 in gfx9's encoding), placed where only
// loads are outstanding; the compiler's waitcnt pass sees the builtin and drops later waits.
__device__ __forceinline__ void wait_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// ---- state I/O -----------------------------------------------------------------------------------
// Addressing: a wave's accesses are a wave-uniform base (field f0 of a channel: ch * n + f0, in SGPRs)
// plus the lane's 32-bit byte offset, so they compile to `global_load/store v, v_off, s[base]`.
// Written as one int64 index (ch * n + f0 + fl) the compiler formed every address per lane with two
// quarter-rate v_mad_u64_u32 (the multiply by n fused into the divergent add): 46 channel loads and
// 46 stores, ~400 VALU slots per wave.  (Laundering the base through readfirstlane spilled SGPRs and
// measured ~1 us slower per step, profiles/r02_ablate_addressing.log.)
// element at (wave-uniform base) + byte offset
template <class T>
__device__ __forceinline__ T& at(T* base, uint32_t byte_off) {
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return *reinterpret_cast<T*>(reinterpret_cast<B*>(base) + byte_off);
}

// fields f0 + fl (f0 wave-uniform).  The channels are walked with one running per-lane pointer
// advanced by the channel stride (n floats, wave-uniform): one 64-bit add per channel.
__device__ __forceinline__ void load_bodies(const float* __restrict__ st, int64_t n, int64_t f0, int fl, Bodies& b) {
  float v[VSS_STATE_CHANNELS];
  const float* q = st + f0 + fl;
#pragma unroll
  for (int c = 0; c < VSS_STATE_CHANNELS; ++c) {
    if (c < VSS_CH_RQX || c >= VSS_CH_RQZ)  // the quaternions' x, y channels are not live (planar)
      v[c] = *q;
    q += n;
  }
  b.bx = v[VSS_CH_BALL_X]; b.by = v[VSS_CH_BALL_Y]; b.bvx = v[VSS_CH_BALL_VX]; b.bvy = v[VSS_CH_BALL_VY];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    b.x[i] = v[VSS_CH_RX + i]; b.y[i] = v[VSS_CH_RY + i]; b.qz[i] = v[VSS_CH_RQZ + i]; b.qw[i] = v[VSS_CH_RQW + i];
    b.vx[i] = v[VSS_CH_RVX + i]; b.vy[i] = v[VSS_CH_RVY + i]; b.w[i] = v[VSS_CH_RW + i];
  }
}

__device__ __forceinline__ void store_bodies(float* __restrict__ st, int64_t n, int64_t f0, int fl, const Bodies& b) {
  float v[VSS_STATE_CHANNELS];
  v[VSS_CH_BALL_X] = b.bx; v[VSS_CH_BALL_Y] = b.by; v[VSS_CH_BALL_VX] = b.bvx; v[VSS_CH_BALL_VY] = b.bvy;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v[VSS_CH_RX + i] = b.x[i]; v[VSS_CH_RY + i] = b.y[i]; v[VSS_CH_RQZ + i] = b.qz[i]; v[VSS_CH_RQW + i] = b.qw[i];
    v[VSS_CH_RVX + i] = b.vx[i]; v[VSS_CH_RVY + i] = b.vy[i]; v[VSS_CH_RW + i] = b.w[i];
  }
  float* q = st + f0 + fl;
#pragma unroll
  for (int c = 0; c < VSS_STATE_CHANNELS; ++c) {
    if (c < VSS_CH_RQX || c >= VSS_CH_RQZ) *q = v[c];
    q += n;
  }
}

// ---- wave-cooperative AoS <-> per-lane transposes through LDS -----------------------------------
// A wave owns fields [f0, f0 + nv); their W-float records are contiguous in global memory.
template <int W>
__device__ __forceinline__ void coop_load(const float* __restrict__ g, int nv, float* lds, int lane) {
  const int total = nv * W;
  if constexpr (W % 4 == 0) {
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int q = lane; q < total / 4; q += kWave) {
      float4 v = at(g4, 16u * (uint32_t)q);
      int e = q * 4, fl = e / W, k = e - fl * W;
      float* d = lds + fl * kRec + k;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  } else {
    const float2* g2 = reinterpret_cast<const float2*>(g);
    for (int q = lane; q < total / 2; q += kWave) {
      float2 v = at(g2, 8u * (uint32_t)q);
      int e = q * 2, fl = e / W, k = e - fl * W;
      float* d = lds + fl * kRec + k;
      d[0] = v.x; d[1] = v.y;
    }
  }
}

template <int W>
__device__ __forceinline__ void coop_store(float* __restrict__ g, int nv, const float* lds, int lane) {
  const int total = nv * W;
  if constexpr (W % 4 == 0) {
    float4* g4 = reinterpret_cast<float4*>(g);
    for (int q = lane; q < total / 4; q += kWave) {
      int e = q * 4, fl = e / W, k = e - fl * W;
      const float* s = lds + fl * kRec + k;
      at(g4, 16u * (uint32_t)q) = make_float4(s[0], s[1], s[2], s[3]);
    }
  } else {
    float2* g2 = reinterpret_cast<float2*>(g);
    for (int q = lane; q < total / 2; q += kWave) {
      int e = q * 2, fl = e / W, k = e - fl * W;
      const float* s = lds + fl * kRec + k;
      at(g2, 8u * (uint32_t)q) = make_float2(s[0], s[1]);
    }
  }
}

// Observation record of one field into LDS (layout above); A = 6 also writes the mirror slots.
template <int A>
__device__ __forceinline__ void write_obs_record(float* rec, const Bodies& b, const float dof[12]) {
  rec[0] = b.bx; rec[1] = b.by; rec[2] = b.bvx; rec[3] = b.bvy;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float* o = rec + 4 + 9 * r;
    o[0] = b.x[r]; o[1] = b.y[r]; o[2] = b.vx[r]; o[3] = b.vy[r];
    o[4] = b.qw[r] * b.qw[r] - b.qz[r] * b.qz[r];
    o[5] = 2.0f * b.qw[r] * b.qz[r];
    o[6] = b.w[r]; o[7] = dof[2 * r]; o[8] = dof[2 * r + 1];
  }
  if constexpr (A == 6) {
    // negation = sign-bit flip (what mirror_tensor's multiply by -1 gives, incl. -0 for 0)
    float* m = rec + kRec;
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = __uint_as_float(__float_as_uint(rec[k]) ^ 0x80000000u);
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int q = 0; q < 6; ++q)
        m[4 + 6 * r + q] = __uint_as_float(__float_as_uint(rec[4 + 9 * r + q]) ^ 0x80000000u);
  }
}

// Stream the wave's observation block (nv fields x A agents x 52) out of the LDS records: each
// lane walks float4 slots q = lane, lane + 64, ... with its (field, slot) position advanced
// incrementally; four LDS reads per float4 at table-given byte offsets, one 16-B store.  Unrolled
// by kObsUnroll so the LDS latency of U slots overlaps (reads past the last field are clamped to
// the last record and their stores predicated off).
//
// nt: nontemporal stores (profiles/r02_ablate_nt_obs.log).  The wrapped modes' steps are 2-5 %
// faster with both observation streams nontemporal (SA 21.3 -> 20.5 us, CMA 21.5 -> 20.4, DMA
// 28.4 -> 27.7).  The FULL step streams 164 MB of observations per 65,536 fields: while its whole
// footprint fits the 256 MiB Infinity Cache plain stores are best (both streams nontemporal: 11 %
// slower, one: +0.5 %); past it, one stream nontemporal and the other plain is best (131,072
// fields: 74.5 -> 68.4 us; both nontemporal: +1.6 % only), so the host sets StepArgs::nt_obs for
// footprints above the cache size and FULL then streams `obs` nontemporally, `terminal_obs` plain.
// The K-step rollout (K x 175 MB per launch) streams both nontemporally: 36.1 -> 33.3 us per step at
// K = 16 (obs alone: no gain).
constexpr int kObsUnroll = 4;
template <int A>
__device__ __forceinline__ void coop_store_obs(float* __restrict__ out, int nv, const float* lds, const uint32_t* tab,
                                               int lane, bool nt = false) {
  constexpr int Q = 13 * A;  // float4 per field
  constexpr int QD = kWave / Q, QR = kWave % Q;
  constexpr uint32_t RB = 4u * obs_rec<A>();  // record bytes
  const int total = nv * Q;
  const uint32_t rb_last = (uint32_t)(nv - 1) * RB;
  int fl = lane / Q, j4 = lane - fl * Q;
  uint32_t rb = (uint32_t)fl * RB;
  const char* L = reinterpret_cast<const char*>(lds);
  float4* o4 = reinterpret_cast<float4*>(out);
  for (int q0 = lane; q0 < total; q0 += kObsUnroll * kWave) {
    float4 v[kObsUnroll];
#pragma unroll
    for (int u = 0; u < kObsUnroll; ++u) {
      const uint2 t = reinterpret_cast<const uint2*>(tab)[j4];  // LDS copy of kObsTab (stage_obs_table)
      const uint32_t r = rb < rb_last ? rb : rb_last;
      v[u].x = *reinterpret_cast<const float*>(L + r + (t.x & 0xffffu));
      v[u].y = *reinterpret_cast<const float*>(L + r + (t.x >> 16));
      v[u].z = *reinterpret_cast<const float*>(L + r + (t.y & 0xffffu));
      v[u].w = *reinterpret_cast<const float*>(L + r + (t.y >> 16));
      j4 += QR;
      rb += QD * RB;
      if (j4 >= Q) { j4 -= Q; rb += RB; }
    }
#pragma unroll
    for (int u = 0; u < kObsUnroll; ++u)
      if (q0 + u * kWave < total) {
        if (nt) {  // wave-uniform
          typedef float f4v __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(f4v{v[u].x, v[u].y, v[u].z, v[u].w},
                                      reinterpret_cast<f4v*>(&at(o4, 16u * (uint32_t)(q0 + u * kWave))));
        } else {
          at(o4, 16u * (uint32_t)(q0 + u * kWave)) = v[u];
        }
      }
  }
}

// ---- reset sampling (envs/vss.py:267-333) --------------------------------------------------------------
// Where the draws come from.  Product: Philox words, counter (field, ctr, purpose << 24 | round, block),
// turned into U[0,1) by u01.  Replay (the parity entries vss_step_replay / vss_reset_dones_replay):
// the field's row of recorded reference draws, `u[14 r + j]` = draw j of rejection round r (one
// (7, 2) row of torch.rand((len(close_ids), 7, 2)), envs/vss.py:283-291), then at 14 R (R = rounds
// used) the 6 yaw draws (torch_rand_float(-pi, pi, (n, 6)), envs/vss.py:307-312) and the 2 ball-
// velocity draws (torch.rand((n, 2)), envs/vss.py:318-325).  A replayed word is the float's bit
// pattern and its conversion the identity, so both sources run the same code below.
struct ResetDraws {
  uint32_t k0, k1, field, ctr, ext;
  const float* u;  // replay: this field's row; product: unused
  uint32_t rounds; // rejection rounds allowed (the replay row's capacity, else kMaxRejectRounds)
};

template <bool REPLAY>
__device__ __forceinline__ float uval(uint32_t w) { return REPLAY ? __uint_as_float(w) : u01(w); }

template <bool REPLAY>
__device__ __forceinline__ void pos_block(const ResetDraws& d, uint32_t round, uint32_t blk, uint32_t o[4]) {
  if constexpr (REPLAY) {
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t j = 4u * blk + i;  // 14 draws per round: the 8th "entity" of block 3 is padding
      o[i] = j < 14u ? __float_as_uint(d.u[14u * round + j]) : 0x3f000000u;
    }
  } else {
    philox(d.k0, d.k1, d.field, d.ctr, ((kPurposePos | d.ext) << 24) | round, blk, o);
  }
}

template <bool REPLAY>
__device__ __forceinline__ void ang_block(const ResetDraws& d, uint32_t rounds_used, uint32_t blk, uint32_t o[4]) {
  if constexpr (REPLAY) {
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) o[i] = __float_as_uint(d.u[14u * rounds_used + 4u * blk + i]);
  } else {
    philox(d.k0, d.k1, d.field, d.ctr, ((kPurposeAng | d.ext) << 24), blk, o);
  }
}

template <bool REPLAY>
__device__ __forceinline__ void reset_field(Bodies& b, const ResetDraws& d) {
  const float scale_x = 1.5f - 0.14f, scale_y = 1.3f - 0.14f;
  float px[7], py[7];
  uint32_t round = 0;
  for (;; ++round) {
    uint32_t o[16];
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) pos_block<REPLAY>(d, round, (uint32_t)blk, o + 4 * blk);
#pragma unroll
    for (int e = 0; e < 7; ++e) {
      px[e] = (uval<REPLAY>(o[2 * e]) - 0.5f) * scale_x;
      py[e] = (uval<REPLAY>(o[2 * e + 1]) - 0.5f) * scale_y;
    }
    bool close = false;
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = i + 1; j < 7; ++j) {
        float dx = px[i] - px[j], dy = py[i] - py[j];
        close |= dx * dx + dy * dy < __uint_as_float(0x3ba0902du);  // == sqrtf(d2) < 0.07f (see below)
      }
    if (!close || round + 1 >= d.rounds) break;
  }
  b.bx = px[0]; b.by = py[0];
  uint32_t o[8];
  ang_block<REPLAY>(d, round + 1, 0u, o);
  ang_block<REPLAY>(d, round + 1, 1u, o + 4);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    b.x[r] = px[1 + r]; b.y[r] = py[1 + r];
    b.vx[r] = 0.0f; b.vy[r] = 0.0f; b.w[r] = 0.0f;
    float ang = K_TWO_PI * uval<REPLAY>(o[r]) + (-K_PI);
    float sh, ch;
    sincos_small(ang * 0.5f, sh, ch);
    float nrm = sqrtf(sh * sh + ch * ch);
    b.qz[r] = sh / nrm;
    b.qw[r] = ch / nrm;
  }
  b.bvx = uval<REPLAY>(o[6]) - 0.5f;
  b.bvy = uval<REPLAY>(o[7]) - 0.5f;
}

// The same reset with the field's two lane halves (L, L + 32) sharing the work: each half draws
// two of the four position blocks and one of the two angle blocks, the values are exchanged with
// v_permlane32_swap, and each half builds three of the six yaw quaternions.  The placement test
// compares squared distances with kMinDist2, the smallest float whose correctly rounded sqrtf is
// >= 0.07f, so `d2 < kMinDist2` is exactly `sqrtf(d2) < 0.07f` (what reset_field and the oracle
// evaluate) without the square roots.  Identical values in every lane to reset_field().
template <bool REPLAY>
__device__ __forceinline__ void reset_field_split(Bodies& b, const ResetDraws& d) {
  const float kMinDist2 = __uint_as_float(0x3ba0902du);  // 0.0048999996f (tests/test_oracle_golden.py)
  const bool up = threadIdx.x >= 32;
  const uint32_t blk0 = up ? 2u : 0u;
  const float scale_x = 1.5f - 0.14f, scale_y = 1.3f - 0.14f;
  float px[8], py[8];
  uint32_t round = 0;
  for (;; ++round) {
    uint32_t o[8];
    pos_block<REPLAY>(d, round, blk0, o);
    pos_block<REPLAY>(d, round, blk0 + 1u, o + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // entities e (lower half) and 4 + e (upper half)
      exch((uval<REPLAY>(o[2 * e]) - 0.5f) * scale_x, px[e], px[4 + e]);
      exch((uval<REPLAY>(o[2 * e + 1]) - 0.5f) * scale_y, py[e], py[4 + e]);
    }
    bool close = false;
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = i + 1; j < 7; ++j) {
        float dx = px[i] - px[j], dy = py[i] - py[j];
        close |= dx * dx + dy * dy < kMinDist2;
      }
    if (!close || round + 1 >= d.rounds) break;
  }
  b.bx = px[0]; b.by = py[0];
  uint32_t oa[4], ang_u[8];
  ang_block<REPLAY>(d, round + 1, up ? 1u : 0u, oa);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float lo, hi;
    exch(__uint_as_float(oa[i]), lo, hi);
    ang_u[i] = __float_as_uint(lo);
    ang_u[4 + i] = __float_as_uint(hi);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {  // robots k (lower half) and k + 3 (upper half)
    float ang = K_TWO_PI * uval<REPLAY>(up ? ang_u[k + 3] : ang_u[k]) + (-K_PI);
    float sh, ch;
    sincos_small(ang * 0.5f, sh, ch);
    float nrm = sqrtf(sh * sh + ch * ch);
    exch(sh / nrm, b.qz[k], b.qz[k + 3]);
    exch(ch / nrm, b.qw[k], b.qw[k + 3]);
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    b.x[r] = px[1 + r]; b.y[r] = py[1 + r];
    b.vx[r] = 0.0f; b.vy[r] = 0.0f; b.w[r] = 0.0f;
  }
  b.bvx = uval<REPLAY>(ang_u[6]) - 0.5f;
  b.bvy = uval<REPLAY>(ang_u[7]) - 0.5f;
}

// ---- rewards and dones (compute_rewards_and_dones, envs/vss.py:218-265, 578-655) --------------------
// (pbx, pby, prx, pry): positions before the physics; `a`: the clamped actions (= dof_velocity_buf).
__device__ __forceinline__ int64_t rewards_and_done(const vss_params& p, const Bodies& b, float pbx, float pby,
                                                   const float prx[6], const float pry[6], const float a[12],
                                                   int64_t progress, float rew[24]) {
  const float bx = b.bx, by = b.by;
  const bool is_goal = (fabsf(bx) > K_FIELD_HX) && (fabsf(by) < K_GOAL_HY);
  const float g = is_goal ? (bx > 0.0f ? 1.0f : (bx < 0.0f ? -1.0f : 0.0f)) : 0.0f;
  float grad;
  {
    float lx = bx - (-K_FIELD_HX), ly = by - (-0.0f), rx = bx - K_FIELD_HX, ry = by - 0.0f;
    float pot = sqrtf(lx * lx + ly * ly) - sqrtf(rx * rx + ry * ry);
    float plx = pbx - (-K_FIELD_HX), ply = pby - (-0.0f), prx_ = pbx - K_FIELD_HX, pry_ = pby - 0.0f;
    float ppot = sqrtf(plx * plx + ply * ply) - sqrtf(prx_ * prx_ + pry_ * pry_);
    grad = pot - ppot;
  }
#pragma unroll
  for (int ag = 0; ag < 6; ++ag) {
    const bool blue = ag < 3;
    float r0 = 0.0f, r1 = 0.0f, r2 = 0.0f, r3 = 0.0f;
    if (p.w_goal > 0.0f) r0 = (blue ? g : (0.0f - g)) * p.w_goal;
    if (p.w_grad > 0.0f) r1 = (blue ? grad : -grad) * p.w_grad;
    if (p.w_move > 0.0f) {
      float dx0 = prx[ag] - pbx, dy0 = pry[ag] - pby;
      float dx1 = b.x[ag] - bx, dy1 = b.y[ag] - by;
      float pd = sqrtf(dx0 * dx0 + dy0 * dy0), d = sqrtf(dx1 * dx1 + dy1 * dy1);
      r2 = 0.0f + (pd - d) * p.w_move;
    }
    if (p.w_energy > 0.0f)
      r3 = 0.0f + (-((fabsf(a[2 * ag]) + fabsf(a[2 * ag + 1])) / 2.0f)) * p.w_energy;
    rew[4 * ag] = r0; rew[4 * ag + 1] = r1; rew[4 * ag + 2] = r2; rew[4 * ag + 3] = r3;
  }
  return (is_goal || progress >= (int64_t)p.max_episode_length) ? 1 : 0;
}

__device__ __forceinline__ void prefetch12(const float* __restrict__ g, int nv, int lane, float4 pre[3]) {
  const float4* g4 = reinterpret_cast<const float4*>(g);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int q = lane + j * kWave;
    if (q < nv * 3) pre[j] = at(g4, 16u * (uint32_t)q);
  }
}

__device__ __forceinline__ void stage12(const float4 pre[3], int nv, float* lds, int lane) {
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int q = lane + j * kWave;
    if (q < nv * 3) {
      const int fl = q / 3, k = (q - fl * 3) * 4;
      float* d = lds + fl * kRec + k;
      d[0] = pre[j].x; d[1] = pre[j].y; d[2] = pre[j].z; d[3] = pre[j].w;
    }
  }
}

// The learner action rows (nv, NL) of a wrapped-mode batch as float2 pieces (8-B aligned per the
// ABI), prefetched into registers and later staged into the LDS record layout like stage12.
template <int NL>
__device__ __forceinline__ void prefetch_lrn(const float* __restrict__ g, int nv, int lane, float2 pre[2]) {
  const float2* g2 = reinterpret_cast<const float2*>(g);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = lane + j * kWave;
    if (q < nv * NL / 2) pre[j] = at(g2, 8u * (uint32_t)q);
  }
}

template <int NL>
__device__ __forceinline__ void stage_lrn(const float2 pre[2], int nv, float* lds, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = lane + j * kWave;
    if (q < nv * NL / 2) {
      const int e = q * 2, fl = e / NL, k = e - fl * NL;
      float* d = lds + fl * kRec + k;
      d[0] = pre[j].x; d[1] = pre[j].y;
    }
  }
}

// random_ou's normals for the wrapped modes with the field's two lane halves sharing the work
// (physics_split's lane pairing): each half draws the Philox blocks and Box-Muller pairs of its
// share of the opponent slots, and v_permlane32_swap gives every lane all of them.  SA (slots
// 2-11: pairs from blocks 0.h1, 1.h0, 1.h1, 2.h0, 2.h1): the lower half takes blocks 0-1, the upper
// block 2; CMA/DMA (slots 6-11: 1.h1, 2.h0, 2.h1): the lower half block 1, the upper block 2.  The
// same operations per pair as the unsplit loop in step_kernel (bit-identical results), about a
// third fewer VALU instructions per wave.
__device__ __forceinline__ void box_muller(uint32_t w1, uint32_t w2, float& zc, float& zs) {
  const float u1 = u01_open0(w1), u2 = u01(w2);
  const float rad = sqrtf(-2.0f * logf_poly(u1));
  float sz, cz;
  sincos_turn(u2, sz, cz);
  zc = K_OU_SIGMA * (rad * cz);
  zs = K_OU_SIGMA * (rad * sz);
}

template <int MODE>
__device__ __forceinline__ void ou_noise_split(float a[12], uint32_t k0, uint32_t k1, uint32_t field, uint32_t ctr) {
  const bool up = threadIdx.x >= 32;
  float z[12];
  if constexpr (MODE == VSS_MODE_SA) {
    uint32_t p[4], q[4];
    philox(k0, k1, field, ctr, kPurposeOU << 24, up ? 2u : 0u, p);
    philox(k0, k1, field, ctr, kPurposeOU << 24, up ? 2u : 1u, q);
    float c0, s0, c1, s1, c2, s2;
    box_muller(up ? p[0] : p[2], up ? p[1] : p[3], c0, s0);  // lower: slots 2,3   upper: 8,9
    box_muller(up ? p[2] : q[0], up ? p[3] : q[1], c1, s1);  // lower: slots 4,5   upper: 10,11
    box_muller(q[2], q[3], c2, s2);                          // lower: slots 6,7   (upper: unused)
    exch(c0, z[2], z[8]);
    exch(s0, z[3], z[9]);
    exch(c1, z[4], z[10]);
    exch(s1, z[5], z[11]);
    float unused;
    exch(c2, z[6], unused);
    exch(s2, z[7], unused);
  } else {
    uint32_t p[4];
    philox(k0, k1, field, ctr, kPurposeOU << 24, up ? 2u : 1u, p);
    float c0, s0, c1, s1;
    box_muller(up ? p[0] : p[2], up ? p[1] : p[3], c0, s0);  // lower: slots 6,7   upper: 8,9
    box_muller(p[2], p[3], c1, s1);                          // (lower: unused)    upper: 10,11
    exch(c0, z[6], z[8]);
    exch(s0, z[7], z[9]);
    float unused;
    exch(c1, unused, z[10]);
    exch(s1, unused, z[11]);
  }
  constexpr int NL = MODE == VSS_MODE_SA ? 2 : 6;
#pragma unroll
  for (int k = NL; k < 12; ++k) a[k] = clampf((a[k] - K_OU_THETA * a[k]) + z[k], -1.0f, 1.0f);
}

// ---- the step kernel -------------------------------------------------------------------------------
// One wave's inputs (kFpw fields), all issued at the start of the kernel: the field's bookkeeping and
// 46 live state channels, and the wave's contiguous AoS blocks of the batch's 12-float action rows
// (FULL) or OU buffer rows (wrapped) and learner action rows (wrapped).
struct BatchIn {
  int64_t progress, reset_prev;
  uint32_t ctr;
  Bodies b;
  float4 blk[3];  // (nv, 12) block: float4 q = lane + 64 j, q < 3 nv
  float2 lrn[2];  // (nv, NL) block: float2 q = lane + 64 j, q < nv NL / 2
};

struct StepArgs {
  int64_t n;
  vss_params p;
  vss_state s;
  vss_step_io io;
  vss_replay_draws rd;  // REPLAY instantiations only (vss_step_replay)
  uint32_t rd_rounds;   // rejection rounds one replay row holds
  uint32_t nt_obs;      // FULL: stream obs with nontemporal stores (footprint past the Infinity Cache)
};

// REPLAY = false: the product kernel (Philox draws).  REPLAY = true: the parity entry
// vss_step_replay, the same kernel consuming recorded reference draws (ResetDraws above; OU
// normals from rd.normals) -- every other instruction is shared.
template <int MODE>
__device__ __forceinline__ void load_batch(const StepArgs& args, int64_t f0, int nv, int fl, int lane, BatchIn& in) {
  constexpr int NL = MODE == VSS_MODE_SA ? 2 : 6;
  in.progress = 0;
  in.reset_prev = 0;
  in.ctr = 0;
  in.b = {};
  if (fl < nv) {
    in.progress = at(args.s.progress_buf + f0, 8u * (uint32_t)fl);
    in.reset_prev = at(args.s.reset_buf + f0, 8u * (uint32_t)fl);
    in.ctr = at(args.s.rng_counter + f0, 4u * (uint32_t)fl);
    load_bodies(args.s.state, args.n, f0, fl, in.b);
  }
  prefetch12((MODE == VSS_MODE_FULL ? args.io.actions : args.io.ou_buf) + f0 * 12, nv, lane, in.blk);
  if constexpr (MODE != VSS_MODE_FULL) prefetch_lrn<NL>(args.io.actions + f0 * NL, nv, lane, in.lrn);
}

template <int MODE, bool REPLAY = false>
__global__ __launch_bounds__(kWave) void step_kernel(StepArgs args) {
  constexpr int A = MODE == VSS_MODE_FULL ? 6 : (MODE == VSS_MODE_DMA ? 3 : 1);
  constexpr int R = MODE == VSS_MODE_DMA ? 3 : 1;
  constexpr int NL = MODE == VSS_MODE_SA ? 2 : 6;  // learner action floats per field
  // lanes L and L + 32 hold field L (physics_split); lanes < 32 address the LDS records, so LDS holds
  // 32 plain records or kFpw observation records, whichever is larger
  static_assert(2 * kFpw == kWave, "two lanes per field");
  constexpr int kLds = 32 * kRec > kFpw * obs_rec<A>() ? 32 * kRec : kFpw * obs_rec<A>();
  static_assert(kFpw * obs_rec<A>() <= kLds, "observation records must fit the LDS block");
  __shared__ float lds[kLds + kTabWords];
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds + kLds);
  stage_obs_table(tab, threadIdx.x);

  const int64_t n = args.n;
  const int lane = threadIdx.x;
  const int fl = lane & 31;        // this lane's field within the wave
  const bool writer = lane < 32;   // writes the field's LDS record slots
  const uint32_t k0 = (uint32_t)args.p.seed, k1 = (uint32_t)(args.p.seed >> 32);
  float* rec = lds + fl * kRec;
  float* orec = lds + lane * obs_rec<A>();  // observation record (lanes < kFpw)

  const int64_t f0 = (int64_t)blockIdx.x * kFpw;
  const int nv = (int)(n - f0 < kFpw ? n - f0 : kFpw);
  BatchIn cur;
  load_batch<MODE>(args, f0, nv, fl, lane, cur);
  const int64_t f = f0 + fl;
  const bool valid = fl < nv;
  const bool owner = valid && writer;  // stores the field's outputs

  int64_t progress = cur.progress, reset_prev = cur.reset_prev;
  uint32_t ctr = cur.ctr;
  Bodies b = cur.b;

  // -- actions: FULL reads (N,12); wrapped modes read + update the OU action buffer --------------
  float a[12];
  stage12(cur.blk, nv, lds, lane);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 12; ++k) a[k] = rec[k];
  __syncthreads();

  if constexpr (MODE != VSS_MODE_FULL) {
    // random_ou (envs/wrappers.py:5-19): a <- clamp(a - 0.1 a + N(0, 0.15^2), -1, 1); the learner
    // slots (pairs 0 for SA, 0..2 for CMA/DMA) are overwritten, so their normals are not needed.
    if constexpr (REPLAY) {
      // torch.normal(0, 0.15, (N, 2, 3, 2)) of random_ou: the field's 12 recorded samples
      if (valid) {
        const float* z = args.rd.normals + f * 12;
#pragma unroll
        for (int k = NL; k < 12; ++k) a[k] = clampf((a[k] - K_OU_THETA * a[k]) + z[k], -1.0f, 1.0f);
      }
    } else {
      ou_noise_split<MODE>(a, k0, k1, (uint32_t)f, ctr);
    }
    stage_lrn<NL>(cur.lrn, nv, lds, lane);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NL; ++k) a[k] = rec[k];
    __syncthreads();
  }
  float ou[12];
  if constexpr (MODE != VSS_MODE_FULL) {
#pragma unroll
    for (int k = 0; k < 12; ++k) ou[k] = a[k];
  }

  // -- Ext VecTask.step clamp + pre_physics_step (envs/vss.py:180-187) -----------------------------
  const float clip = args.p.clip_actions;
#pragma unroll
  for (int k = 0; k < 12; ++k) a[k] = clampf(a[k], -clip, clip);
  if (reset_prev != 0) progress = 0;

  float pbx = b.bx, pby = b.by, prx[6], pry[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) { prx[i] = b.x[i]; pry[i] = b.y[i]; }

  // -- gym.simulate replacement ------------------------------------------------------------------------
  if (valid) physics_split(b, a);

  // -- post_physics_step: progress, rewards, dones (envs/vss.py:189-265) ----------------------------------
  progress += 1;
  float rew[24];
  const int64_t done = rewards_and_done(args.p, b, pbx, pby, prx, pry, a, progress, rew);

  // Retire every pending load here, before the first store: gfx9's vmcnt counts loads and stores, and
  // the compiler can only wait for a load issued before stores by draining those stores too -- e.g.
  // the rng counter, first used by the reset.
  wait_loads();

  // -- terminal observation (envs/vss.py:195-196) ----------------------------------------------------------
  if (lane < kFpw) write_obs_record<A>(orec, b, a);
  __syncthreads();
  coop_store_obs<A>(args.io.terminal_obs + f0 * (52 * A), nv, lds, tab, lane, MODE != VSS_MODE_FULL);
  __syncthreads();

  // -- reset_dones (envs/vss.py:202, 267-333) ---------------------------------------------------------------
  float dof[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) dof[k] = a[k];
  if (valid && done) {
    const ResetDraws rd{k0, k1, (uint32_t)f, ctr, 0u, REPLAY ? args.rd.uniforms + f * args.rd.uniform_stride : nullptr,
                        REPLAY ? args.rd_rounds : (uint32_t)kMaxRejectRounds};
    reset_field_split<REPLAY>(b, rd);
#pragma unroll
    for (int k = 0; k < 12; ++k) dof[k] = dof[k] * 0.0f;
  }

  // -- observation after reset (envs/vss.py:203) -------------------------------------------------------------
  if (lane < kFpw) write_obs_record<A>(orec, b, dof);
  __syncthreads();
  coop_store_obs<A>(args.io.obs + f0 * (52 * A), nv, lds, tab, lane, MODE != VSS_MODE_FULL || args.nt_obs != 0);
  __syncthreads();

  // -- bookkeeping --------------------------------------------------------------------------------------------
  const uint8_t time_out = (progress >= (int64_t)args.p.max_episode_length - 1) && done != 0;
  if (owner) {
    const uint32_t ufl = (uint32_t)fl;
    store_bodies(args.s.state, n, f0, fl, b);
    at(args.s.progress_buf + f0, 8u * ufl) = progress;
    at(args.s.reset_buf + f0, 8u * ufl) = done;
    at(args.s.rng_counter + f0, 4u * ufl) = ctr + 1u;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      at(args.io.time_outs + f0 * R, (uint32_t)(ufl * R + k)) = time_out;
      at(args.io.progress_f + f0 * R, 4u * (ufl * R + k)) = (float)progress;
    }
    if constexpr (MODE == VSS_MODE_DMA) {
#pragma unroll
      for (int k = 0; k < 3; ++k) at(args.io.dones_rep + f0 * 3, 8u * (ufl * 3 + k)) = done;
    }
  }

  // dof_velocity_buf (N,12) and, wrapped, the OU action buffer (zeroed for done fields)
  if (writer) {
#pragma unroll
    for (int k = 0; k < 12; ++k) rec[k] = dof[k];
  }
  __syncthreads();
  coop_store<12>(args.s.dof_velocity_buf + f0 * 12, nv, lds, lane);
  __syncthreads();
  if constexpr (MODE != VSS_MODE_FULL) {
    if (writer) {
#pragma unroll
      for (int k = 0; k < 12; ++k) rec[k] = done ? ou[k] * 0.0f : ou[k];
    }
    __syncthreads();
    coop_store<12>(args.io.ou_buf + f0 * 12, nv, lds, lane);
    __syncthreads();
  }

  // rewards
  if constexpr (MODE == VSS_MODE_FULL) {
    if (writer) {
#pragma unroll
      for (int k = 0; k < 24; ++k) rec[k] = rew[k];
    }
    __syncthreads();
    coop_store<24>(args.io.rew + f0 * 24, nv, lds, lane);
    if (owner && args.io.reward_sum) at(args.io.reward_sum + f0, 4u * (uint32_t)fl) = ((rew[0] + rew[1]) + rew[2]) + rew[3];
  } else if constexpr (MODE == VSS_MODE_SA) {
    if (owner) {
      at(reinterpret_cast<float4*>(args.io.rew) + f0, 16u * (uint32_t)fl) = make_float4(rew[0], rew[1], rew[2], rew[3]);
      at(args.io.reward_sum + f0, 4u * (uint32_t)fl) = ((rew[0] + rew[1]) + rew[2]) + rew[3];
    }
  } else if constexpr (MODE == VSS_MODE_CMA) {
    if (owner) {
      float m[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) m[c] = ((rew[c] + rew[4 + c]) + rew[8 + c]) / 3.0f;
      at(reinterpret_cast<float4*>(args.io.rew) + f0, 16u * (uint32_t)fl) = make_float4(m[0], m[1], m[2], m[3]);
      at(args.io.reward_sum + f0, 4u * (uint32_t)fl) = ((m[0] + m[1]) + m[2]) + m[3];
    }
  } else {
    if (writer) {
#pragma unroll
      for (int k = 0; k < 12; ++k) rec[k] = rew[k];
    }
    __syncthreads();
    coop_store<12>(args.io.rew + f0 * 12, nv, lds, lane);
    if (owner) {
#pragma unroll
      for (int ag = 0; ag < 3; ++ag)
        at(args.io.reward_sum + f0 * 3, 4u * ((uint32_t)fl * 3 + ag)) =
            ((rew[4 * ag] + rew[4 * ag + 1]) + rew[4 * ag + 2]) + rew[4 * ag + 3];
    }
  }
}

// ---- K control steps per launch (open-loop action sequences) -----------------------------------------
// Same per-step semantics as K consecutive step_kernel<FULL> launches, bit for bit (the Philox
// counter of step k is rng_counter + k), but the field state stays in registers across steps, each
// step's observation stores drain while the next step's physics runs, and the next step's actions
// are prefetched into registers before the current step's streams are issued.
struct RolloutArgs {
  int64_t n;
  int32_t k_steps;
  vss_params p;
  vss_state s;
  vss_rollout_io io;
};

__global__ __launch_bounds__(kWave) void rollout_kernel(RolloutArgs args) {
  static_assert(kFpw * kRecObs6 <= kWave * kRec, "observation records must fit the LDS block");
  __shared__ float lds[kWave * kRec + kTabWords];
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds + kWave * kRec);
  stage_obs_table(tab, threadIdx.x);
  const int64_t n = args.n;
  const int lane = threadIdx.x;
  const int fl = lane & (kFpw - 1);  // lanes L and L + 32 hold the same field
  const int64_t f0 = (int64_t)blockIdx.x * kFpw;
  const int nv = (int)(n - f0 < kFpw ? n - f0 : kFpw);
  const int64_t f = f0 + fl;
  const bool valid = fl < nv;  // both halves carry the state (and apply resets) across steps
  const bool owner = valid && lane < kFpw;
  const bool writer = lane < kFpw;
  const uint32_t k0 = (uint32_t)args.p.seed, k1 = (uint32_t)(args.p.seed >> 32);
  float* rec = lds + fl * kRec;
  float* orec = lds + lane * kRecObs6;  // observation record (lanes < kFpw)

  int64_t progress = 0, reset_prev = 0;
  uint32_t ctr = 0;
  Bodies b = {};
  if (valid) {
    progress = at(args.s.progress_buf + f0, 8u * (uint32_t)fl);
    reset_prev = at(args.s.reset_buf + f0, 8u * (uint32_t)fl);
    ctr = at(args.s.rng_counter + f0, 4u * (uint32_t)fl);
    load_bodies(args.s.state, n, f0, fl, b);
  }
  float4 pre[3];
  prefetch12(args.io.actions + f0 * 12, nv, lane, pre);
  float dof[12];
  int64_t done = reset_prev;
  const float clip = args.p.clip_actions;

  for (int k = 0; k < args.k_steps; ++k) {
    const int64_t step_off = (int64_t)k * n;
    float a[12];
    stage12(pre, nv, lds, lane);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 12; ++i) a[i] = clampf(rec[i], -clip, clip);
    __syncthreads();
    if (k + 1 < args.k_steps) prefetch12(args.io.actions + (step_off + n + f0) * 12, nv, lane, pre);

    if (reset_prev != 0) progress = 0;
    float pbx = b.bx, pby = b.by, prx[6], pry[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) { prx[i] = b.x[i]; pry[i] = b.y[i]; }
    if (valid) {
      physics_split(b, a);
    }
    progress += 1;
    float rew[24];
    done = rewards_and_done(args.p, b, pbx, pby, prx, pry, a, progress, rew);

    // the next step's action prefetch (issued before this step's physics) is retired here, before
    // this step's stores: the previous step's stores, issued before it, have drained behind the
    // physics, and the streams below leave no load pending (see wait_loads)
    wait_loads();
    if (lane < kFpw) write_obs_record<6>(orec, b, a);
    __syncthreads();
    coop_store_obs<6>(args.io.terminal_obs + (step_off + f0) * 312, nv, lds, tab, lane, true);  // K steps: past the cache
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 12; ++i) dof[i] = a[i];
    if (valid && done) {
      const ResetDraws rd{k0, k1, (uint32_t)f, ctr + (uint32_t)k, 0u, nullptr, (uint32_t)kMaxRejectRounds};
      reset_field_split<false>(b, rd);
#pragma unroll
      for (int i = 0; i < 12; ++i) dof[i] = dof[i] * 0.0f;
    }
    if (lane < kFpw) write_obs_record<6>(orec, b, dof);
    __syncthreads();
    coop_store_obs<6>(args.io.obs + (step_off + f0) * 312, nv, lds, tab, lane, true);
    __syncthreads();
    if (writer) {
#pragma unroll
      for (int i = 0; i < 24; ++i) rec[i] = rew[i];
    }
    __syncthreads();
    coop_store<24>(args.io.rew + (step_off + f0) * 24, nv, lds, lane);
    __syncthreads();
    if (owner) {
      args.io.dones[step_off + f] = done;
      args.io.time_outs[step_off + f] = (progress >= (int64_t)args.p.max_episode_length - 1) && done != 0;
      args.io.progress_f[step_off + f] = (float)progress;
    }
    reset_prev = done;
  }

  if (owner) {
    store_bodies(args.s.state, n, f0, fl, b);
    args.s.progress_buf[f] = progress;
    args.s.reset_buf[f] = done;
    args.s.rng_counter[f] = ctr + (uint32_t)args.k_steps;
  }
  if (writer) {
#pragma unroll
    for (int i = 0; i < 12; ++i) rec[i] = dof[i];
  }
  __syncthreads();
  coop_store<12>(args.s.dof_velocity_buf + f0 * 12, nv, lds, lane);
}

// External reset_dones: fields with reset_buf != 0 are re-sampled with the EXTERNAL purpose bit
// and their rng counter advances (so repeated calls draw afresh).  dof_velocity_buf zeroed.
// REPLAY: vss_reset_dones_replay, the recorded reference draws instead of Philox.
template <bool REPLAY>
__global__ __launch_bounds__(kWave) void reset_kernel(int64_t n, vss_params p, vss_state s, vss_replay_draws rdr,
                                                     uint32_t rounds) {
  const int64_t f = (int64_t)blockIdx.x * kWave + threadIdx.x;
  if (f >= n || s.reset_buf[f] == 0) return;
  Bodies b;
  const int64_t f0 = (int64_t)blockIdx.x * kWave;
  load_bodies(s.state, n, f0, (int)threadIdx.x, b);
  const uint32_t ctr = s.rng_counter[f];
  const ResetDraws rd{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), (uint32_t)f, ctr, kExternal,
                      REPLAY ? rdr.uniforms + f * rdr.uniform_stride : nullptr, REPLAY ? rounds : (uint32_t)kMaxRejectRounds};
  reset_field<REPLAY>(b, rd);
  store_bodies(s.state, n, f0, (int)threadIdx.x, b);
  s.rng_counter[f] = ctr + 1u;
#pragma unroll
  for (int k = 0; k < 12; ++k) s.dof_velocity_buf[f * 12 + k] = s.dof_velocity_buf[f * 12 + k] * 0.0f;
}

template <int A>
__global__ __launch_bounds__(kWave) void observe_kernel(int64_t n, vss_state s, float* obs) {
  __shared__ float lds[kWave * obs_rec<A>() + kTabWords];
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds + kWave * obs_rec<A>());
  stage_obs_table(tab, threadIdx.x);
  const int lane = threadIdx.x;
  const int64_t f0 = (int64_t)blockIdx.x * kWave;
  const int nv = (int)(n - f0 < kWave ? n - f0 : kWave);

  float* rec = lds + lane * kRec;
  float* orec = lds + lane * obs_rec<A>();
  coop_load<12>(s.dof_velocity_buf + f0 * 12, nv, lds, lane);
  __syncthreads();
  float dof[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) dof[k] = rec[k];
  __syncthreads();
  Bodies b = {};
  if (lane < nv) {
    load_bodies(s.state, n, f0, lane, b);
    write_obs_record<A>(orec, b, dof);
  }
  wait_loads();
  __syncthreads();
  coop_store_obs<A>(obs + f0 * (52 * A), nv, lds, tab, lane);
}

// RecordEpisodeStatisticsTorch.step (envs/wrappers.py:66-87), one row per lane.  The products
// by (1 - done) keep torch's float semantics: x * 0 = -0 for negative x.
__global__ __launch_bounds__(256) void episode_stats_kernel(int64_t rows, const float4* __restrict__ rews,
                                                            const int64_t* __restrict__ dones, float4* ep_ret,
                                                            int32_t* ep_len, float4* __restrict__ ret_out,
                                                            int32_t* __restrict__ len_out, float* __restrict__ sum_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const float4 r = rews[i];
  float4 e = ep_ret[i];
  e.x = e.x + r.x; e.y = e.y + r.y; e.z = e.z + r.z; e.w = e.w + r.w;
  const int32_t l = ep_len[i] + 1;
  ret_out[i] = e;
  len_out[i] = l;
  sum_out[i] = ((e.x + e.y) + e.z) + e.w;
  const int64_t keep = 1 - dones[i];
  const float kf = (float)keep;
  ep_ret[i] = make_float4(e.x * kf, e.y * kf, e.z * kf, e.w * kf);
  ep_len[i] = (int32_t)(l * keep);
}

}  // namespace vss

// ================================================================================================
// C ABI
// ================================================================================================
// Null or misaligned: the kernels move float4 / float2 vectors and int64 scalars.
static bool bad(const void* ptr, uintptr_t align) { return !ptr || (reinterpret_cast<uintptr_t>(ptr) & (align - 1)); }
static bool misaligned(const void* ptr, uintptr_t align) { return ptr && (reinterpret_cast<uintptr_t>(ptr) & (align - 1)); }

static int check_state(int64_t n, const vss_state* st) {
  if (n < 0 || n > (int64_t(1) << 26) || !st) return VSS_E_ARG;
  if (bad(st->state, 4) || bad(st->progress_buf, 8) || bad(st->reset_buf, 8) || bad(st->dof_velocity_buf, 16) ||
      bad(st->rng_counter, 4))
    return VSS_E_ARG;
  return VSS_OK;
}

static int launch_status() { return hipGetLastError() == hipSuccess ? VSS_OK : VSS_E_LAUNCH; }

// Rejection rounds one replay row holds: (stride - 8) / 14.  A row with more rounds than the kernel
// bounds (kMaxRejectRounds) is refused here rather than replayed short (the kernel would stop early
// and read round draws as yaw draws).
static int replay_rounds(const vss_replay_draws* d) {
  if (!d || bad(d->uniforms, 4) || d->uniform_stride < 22 || d->uniform_stride > (int64_t(1) << 20)) return -1;
  const int64_t r = (d->uniform_stride - 8) / 14;
  return r > vss::kMaxRejectRounds ? -1 : (int)r;
}

template <bool REPLAY>
static int step_impl(void* stream, int64_t n, int32_t mode, const vss_params* p, const vss_state* st,
                     const vss_step_io* io, const vss_replay_draws* rd) {
  if (int rc = check_state(n, st)) return rc;
  if (!p || !io || mode < VSS_MODE_FULL || mode > VSS_MODE_DMA) return VSS_E_ARG;
  if (bad(io->actions, mode == VSS_MODE_FULL ? 16 : 8) || bad(io->obs, 16) || bad(io->terminal_obs, 16) ||
      bad(io->rew, 16) || bad(io->time_outs, 1) || bad(io->progress_f, 4) || misaligned(io->reward_sum, 4) ||
      misaligned(io->ou_buf, 16) || misaligned(io->dones_rep, 8))
    return VSS_E_ARG;
  if (mode != VSS_MODE_FULL && (!io->ou_buf || !io->reward_sum)) return VSS_E_ARG;
  if (mode == VSS_MODE_DMA && !io->dones_rep) return VSS_E_ARG;
  int rounds = 0;
  if (REPLAY) {
    rounds = replay_rounds(rd);
    if (rounds < 1 || (mode != VSS_MODE_FULL && bad(rd->normals, 4))) return VSS_E_ARG;
  }
  if (n == 0) return VSS_OK;
  // FULL: the observation stream nontemporal once the step's footprint (3,101 B per field) is past
  // the 256 MiB Infinity Cache (coop_store_obs)
  const uint32_t nt_obs = mode == VSS_MODE_FULL && n > (int64_t)(256ll << 20) / 3101 ? 1u : 0u;
  vss::StepArgs args{n, *p, *st, *io, REPLAY ? *rd : vss_replay_draws{}, (uint32_t)rounds, nt_obs};
  const dim3 grid((unsigned)((n + vss::kFpw - 1) / vss::kFpw)), block(vss::kWave);
  hipStream_t s = (hipStream_t)stream;
  switch (mode) {
    case VSS_MODE_FULL: hipLaunchKernelGGL((vss::step_kernel<VSS_MODE_FULL, REPLAY>), grid, block, 0, s, args); break;
    case VSS_MODE_SA: hipLaunchKernelGGL((vss::step_kernel<VSS_MODE_SA, REPLAY>), grid, block, 0, s, args); break;
    case VSS_MODE_CMA: hipLaunchKernelGGL((vss::step_kernel<VSS_MODE_CMA, REPLAY>), grid, block, 0, s, args); break;
    default: hipLaunchKernelGGL((vss::step_kernel<VSS_MODE_DMA, REPLAY>), grid, block, 0, s, args); break;
  }
  return launch_status();
}

extern "C" {

int vss_abi_version(void) { return VSS_ABI_VERSION; }


const char* vss_error_string(int code) {
  switch (code) {
    case VSS_OK: return "ok";
    case VSS_E_ARG: return "invalid argument (null or misaligned buffer, bad size or bad mode)";
    case VSS_E_LAUNCH: return "kernel launch failed";
    default: return "unknown error";
  }
}

int vss_step(void* stream, int64_t n, int32_t mode, const vss_params* p, const vss_state* st,
             const vss_step_io* io) {
  return step_impl<false>(stream, n, mode, p, st, io, nullptr);
}

int vss_step_replay(void* stream, int64_t n, int32_t mode, const vss_params* p, const vss_state* st,
                    const vss_step_io* io, const vss_replay_draws* draws) {
  return step_impl<true>(stream, n, mode, p, st, io, draws);
}

int vss_rollout(void* stream, int64_t n, int32_t k_steps, const vss_params* p, const vss_state* st,
                const vss_rollout_io* io) {
  if (int rc = check_state(n, st)) return rc;
  if (!p || !io || k_steps < 1 || k_steps > (1 << 20)) return VSS_E_ARG;
  if (bad(io->actions, 16) || bad(io->obs, 16) || bad(io->terminal_obs, 16) || bad(io->rew, 16) ||
      bad(io->dones, 8) || bad(io->time_outs, 1) || bad(io->progress_f, 4))
    return VSS_E_ARG;
  if (n == 0) return VSS_OK;
  vss::RolloutArgs args{n, k_steps, *p, *st, *io};
  const dim3 grid((unsigned)((n + vss::kFpw - 1) / vss::kFpw)), block(vss::kWave);
  hipLaunchKernelGGL(vss::rollout_kernel, grid, block, 0, (hipStream_t)stream, args);
  return launch_status();
}

int vss_reset_dones(void* stream, int64_t n, const vss_params* p, const vss_state* st) {
  if (int rc = check_state(n, st)) return rc;
  if (!p) return VSS_E_ARG;
  if (n == 0) return VSS_OK;
  const dim3 grid((unsigned)((n + vss::kWave - 1) / vss::kWave)), block(vss::kWave);
  hipLaunchKernelGGL(vss::reset_kernel<false>, grid, block, 0, (hipStream_t)stream, n, *p, *st, vss_replay_draws{},
                     (uint32_t)vss::kMaxRejectRounds);
  return launch_status();
}

int vss_reset_dones_replay(void* stream, int64_t n, const vss_params* p, const vss_state* st,
                           const vss_replay_draws* draws) {
  if (int rc = check_state(n, st)) return rc;
  const int rounds = replay_rounds(draws);
  if (!p || rounds < 1) return VSS_E_ARG;
  if (n == 0) return VSS_OK;
  const dim3 grid((unsigned)((n + vss::kWave - 1) / vss::kWave)), block(vss::kWave);
  hipLaunchKernelGGL(vss::reset_kernel<true>, grid, block, 0, (hipStream_t)stream, n, *p, *st, *draws,
                     (uint32_t)rounds);
  return launch_status();
}

int vss_compute_observations(void* stream, int64_t n, const vss_state* st, float* obs, int32_t n_agents) {
  if (int rc = check_state(n, st)) return rc;
  if (bad(obs, 16) || !(n_agents == 1 || n_agents == 3 || n_agents == 6)) return VSS_E_ARG;
  if (n == 0) return VSS_OK;
  const dim3 grid((unsigned)((n + vss::kWave - 1) / vss::kWave)), block(vss::kWave);
  hipStream_t s = (hipStream_t)stream;
  if (n_agents == 6) hipLaunchKernelGGL(vss::observe_kernel<6>, grid, block, 0, s, n, *st, obs);
  else if (n_agents == 3) hipLaunchKernelGGL(vss::observe_kernel<3>, grid, block, 0, s, n, *st, obs);
  else hipLaunchKernelGGL(vss::observe_kernel<1>, grid, block, 0, s, n, *st, obs);
  return launch_status();
}

int vss_episode_stats(void* stream, int64_t rows, const float* rews, const int64_t* dones, float* ep_returns,
                      int32_t* ep_lengths, float* returned_returns, int32_t* returned_lengths, float* return_sum) {
  if (rows < 0 || rows > (int64_t(1) << 31) || bad(rews, 16) || bad(dones, 8) || bad(ep_returns, 16) ||
      bad(ep_lengths, 4) || bad(returned_returns, 16) || bad(returned_lengths, 4) || bad(return_sum, 4))
    return VSS_E_ARG;
  if (rows == 0) return VSS_OK;
  const dim3 grid((unsigned)((rows + 255) / 256)), block(256);
  hipLaunchKernelGGL(vss::episode_stats_kernel, grid, block, 0, (hipStream_t)stream, rows,
                     reinterpret_cast<const float4*>(rews), dones, reinterpret_cast<float4*>(ep_returns), ep_lengths,
                     reinterpret_cast<float4*>(returned_returns), returned_lengths, return_sum);
  return launch_status();
}

}  // extern "C"
