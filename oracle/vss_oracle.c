/*
 * vss_oracle.c — TEST INFRASTRUCTURE ONLY (see vss_oracle.h).
 *
 * Plain-C, single-thread, float32 restatement of the reference's VSS step.  Each function
 * cites the reference file:line it follows (paths relative to the reference repository).
 * The physics section restates the build's own 2D model; no reference code
 * exists for it (PhysX, Ext).  Compile with -ffp-contract=off: the HIP kernel is compiled the
 * same way, so the two agree bit for bit.
 */
#include "vss_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Constants.  Reference values: envs/vss.py:48-49 (42 rad/s, 0.07 m), 342-345 (field),
 * envs/vss.yaml:6-16, envs/vss_robot.urdf (robot).  Model constants: DESIGN.md §3.
 * ---------------------------------------------------------------------------------------- */
#define O_NSUB 2
#define O_H 0.025f            /* dt / NSUB, dt = 0.05 (envs/vss.yaml:16); 2 substeps as Isaac Gym */
#define O_HH 0.0125f          /* H / 2 (half-angle step)                 */
#define O_FIELD_HX 0.75f      /* field_width / 2  (envs/vss.py:343)      */
#define O_FIELD_HY 0.65f      /* field_height / 2                        */
#define O_GOAL_HY 0.2f        /* goal_height / 2  (envs/vss.py:344)      */
#define O_GOAL_BACK_X 0.85f   /* field_width/2 + goal_width              */
#define O_BALL_R 0.02134f     /* envs/vss.py:383                         */
#define O_BALL_R2 0.00045539559f
#define O_ROBOT_HALF 0.035f   /* 0.07 box, envs/vss_robot.urdf:13        */
#define O_ROBOT_R 0.04f       /* disc radius for robot-robot/robot-wall  */
#define O_RR_DIST 0.08f
#define O_RR_DIST2 0.0064f
#define O_WHEEL_RAD_S 42.0f   /* envs/vss.py:48                          */
#define O_WHEEL_R 0.024f      /* envs/vss.py:401                         */
#define O_HALF_TRACK 0.03375f /* envs/vss_robot.urdf:54,62               */
#define O_INV_TRACK 14.814815f
#define O_DV 0.15f            /* wheel traction accel 6 m/s^2 * H        */
#define O_DL 0.171675f        /* lateral friction accel 0.7*9.81 * H     */
#define O_K_BALL 0.99625f     /* ball rolling damping 0.15/s over H      */
#define O_W_ROBOT_BR 0.09465021f /* m_ball / (m_ball + m_robot) */
#define O_W_BALL_BR 0.90534979f  /* m_robot / (m_ball + m_robot) */

#define O_MIN_DIST 0.07f      /* envs/vss.py:49 */
#define O_TWO_PI 6.2831855f
#define O_PI 3.1415927f
#define O_OU_THETA 0.1f       /* envs/wrappers.py:6 */
#define O_OU_SIGMA 0.15f      /* envs/wrappers.py:7 */
#define O_MAX_REJECT_ROUNDS 64

#define O_PURPOSE_OU 1u
#define O_PURPOSE_POS 2u
#define O_PURPOSE_ANG 3u
#define O_EXTERNAL 0x80000000u

#define CH(st, c, n, f) ((st)[(int64_t)(c) * (n) + (f)])

int oracle_abi_version(void) { return VSS_ABI_VERSION; }

/* ------------------------------------------------------------------------------------------
 * Counter-based RNG (Philox4x32-10) and transcendental-free math shared by spec with the
 * kernel.  Not from the reference (torch's generator cannot be matched bit for bit).
 * ---------------------------------------------------------------------------------------- */
void oracle_philox(uint32_t k0, uint32_t k1, const uint32_t ctr[4], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static float u01(uint32_t x) { return (float)(x >> 8) * 5.9604645e-08f; }        /* [0,1) */
static float u01_open0(uint32_t x) { return (float)((x >> 8) + 1u) * 5.9604645e-08f; } /* (0,1] */

static void sincos_poly(float r, float* s, float* c) {
  float r2 = r * r;
  *s = r + r * r2 * (-0.16666667f + r2 * (0.008333334f + r2 * (-1.9841270e-4f + r2 * 2.7557319e-6f)));
  *c = 1.0f + r2 * (-0.5f + r2 * (0.041666668f + r2 * (-1.3888889e-3f + r2 * (2.4801587e-5f + r2 * (-2.7557319e-7f)))));
}

/* sin/cos of x for |x| <= ~3pi/4 (half-angles and small rotation steps). */
void oracle_sincosf(float x, float* s, float* c) {
  if (fabsf(x) < 0.78f) { sincos_poly(x, s, c); return; } /* no reduction needed */
  int k = (int)(x * 0.63661977f + (x >= 0.0f ? 0.5f : -0.5f));
  float kf = (float)k;
  float r = (x - kf * 1.5707964f) - kf * (-4.3711390e-8f);
  float sr, cr;
  sincos_poly(r, &sr, &cr);
  switch (k) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case -1: *s = -cr; *c = sr; break;
    default: *s = -sr; *c = -cr; break; /* k = +-2 */
  }
}

/* cos/sin(2*pi*u), u in [0,1) (Box-Muller angle) */
static void sincos_turn(float u, float* s, float* c) {
  float v = u * 4.0f;
  int q = (int)v;
  float t = v - (float)q;
  float r = (t - 0.5f) * 1.5707964f;
  float sr, cr;
  sincos_poly(r, &sr, &cr);
  float cp = (cr - sr) * 0.70710677f;
  float sp = (cr + sr) * 0.70710677f;
  switch (q) {
    case 0: *c = cp; *s = sp; break;
    case 1: *c = -sp; *s = cp; break;
    case 2: *c = -cp; *s = -sp; break;
    default: *c = sp; *s = -cp; break;
  }
}

float oracle_logf(float x) {
  union { float f; uint32_t u; } b;
  b.f = x;
  int e = (int)((b.u >> 23) & 0xffu) - 127;
  b.u = (b.u & 0x7fffffu) | 0x3f800000u;
  float m = b.f;
  if (m > 1.4142135f) { m = m * 0.5f; e = e + 1; }
  float s = (m - 1.0f) / (m + 1.0f);
  float s2 = s * s;
  float p = 2.0f + s2 * (0.6666667f + s2 * (0.4f + s2 * (0.2857143f + s2 * (0.22222222f + s2 * 0.18181819f))));
  return (float)e * 0.69314718f + s * p;
}

static float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

/* ------------------------------------------------------------------------------------------
 * Draw providers.  Philox mode: counter (field, rng_counter, purpose<<24 | round, block).
 * Injected mode: the recorded torch streams, consumed in the reference's call order.
 * ---------------------------------------------------------------------------------------- */
typedef struct provider {
  const vss_params* p;
  oracle_draws* draws;
} provider;

static float draw_uniform(provider* pv, uint32_t field, uint32_t ctr, uint32_t purpose,
                          uint32_t round, uint32_t k) {
  if (pv->draws) {
    oracle_draws* d = pv->draws;
    if (d->uniform_pos >= d->n_uniforms) return 0.5f; /* exhausted: caller checks cursor */
    return d->uniforms[d->uniform_pos++];
  }
  uint32_t c[4] = {field, ctr, (purpose << 24) | round, k >> 2}, o[4];
  oracle_philox((uint32_t)pv->p->seed, (uint32_t)(pv->p->seed >> 32), c, o);
  return u01(o[k & 3]);
}

/* 12 OU noise samples (already * sigma) for one field, slots in (team, robot, wheel) order */
static void draw_ou_noise(provider* pv, uint32_t field, uint32_t ctr, float out[12]) {
  if (pv->draws) {
    oracle_draws* d = pv->draws;
    for (int k = 0; k < 12; ++k)
      out[k] = d->normal_pos < d->n_normals ? d->normals[d->normal_pos++] : 0.0f;
    return;
  }
  for (uint32_t b = 0; b < 3; ++b) {
    uint32_t c[4] = {field, ctr, O_PURPOSE_OU << 24, b}, o[4];
    oracle_philox((uint32_t)pv->p->seed, (uint32_t)(pv->p->seed >> 32), c, o);
    for (int h = 0; h < 2; ++h) {
      float u1 = u01_open0(o[2 * h]);
      float u2 = u01(o[2 * h + 1]);
      float rad = sqrtf(-2.0f * oracle_logf(u1));
      float sz, cz;
      sincos_turn(u2, &sz, &cz);
      out[4 * b + 2 * h] = O_OU_SIGMA * (rad * cz);
      out[4 * b + 2 * h + 1] = O_OU_SIGMA * (rad * sz);
    }
  }
}

/* ------------------------------------------------------------------------------------------
 * Physics (the build's 2D model; replaces Ext PhysX gym.simulate).  DESIGN.md §3.
 * ---------------------------------------------------------------------------------------- */
typedef struct body_state {
  float bx, by, bvx, bvy;
  float x[6], y[6], qz[6], qw[6], vx[6], vy[6], w[6];
  float c[6], s[6];
} body_state;

static void heading(body_state* b, int i) {
  b->c[i] = b->qw[i] * b->qw[i] - b->qz[i] * b->qz[i];
  b->s[i] = 2.0f * b->qw[i] * b->qz[i];
}

static void contact_robot_robot(body_state* b, int i, int j) {
  float dx = b->x[j] - b->x[i], dy = b->y[j] - b->y[i];
  float d2 = dx * dx + dy * dy;
  if (!(d2 < O_RR_DIST2)) return;
  float d = sqrtf(d2);
  float nx = 1.0f, ny = 0.0f;
  if (d > 1e-9f) { float inv = 1.0f / d; nx = dx * inv; ny = dy * inv; }
  float half = (O_RR_DIST - d) * 0.5f;
  b->x[i] = b->x[i] - nx * half; b->y[i] = b->y[i] - ny * half;
  b->x[j] = b->x[j] + nx * half; b->y[j] = b->y[j] + ny * half;
  float vn = (b->vx[j] - b->vx[i]) * nx + (b->vy[j] - b->vy[i]) * ny;
  if (vn < 0.0f) {
    float jn = vn * 0.5f;
    b->vx[i] = b->vx[i] + nx * jn; b->vy[i] = b->vy[i] + ny * jn;
    b->vx[j] = b->vx[j] - nx * jn; b->vy[j] = b->vy[j] - ny * jn;
  }
}

static void contact_ball_robot(body_state* b, int i) {
  float dx = b->bx - b->x[i], dy = b->by - b->y[i];
  float c = b->c[i], s = b->s[i];
  float lx = c * dx + s * dy;
  float ly = c * dy - s * dx;
  float cx = clampf(lx, -O_ROBOT_HALF, O_ROBOT_HALF);
  float cy = clampf(ly, -O_ROBOT_HALF, O_ROBOT_HALF);
  float ex = lx - cx, ey = ly - cy;
  float d2 = ex * ex + ey * ey;
  float nlx, nly, pen;
  if (d2 > 0.0f) {
    if (!(d2 < O_BALL_R2)) return;
    float d = sqrtf(d2);
    float inv = 1.0f / d;
    nlx = ex * inv; nly = ey * inv;
    pen = O_BALL_R - d;
  } else {
    float px = O_ROBOT_HALF - fabsf(lx), py = O_ROBOT_HALF - fabsf(ly);
    if (px < py) { nlx = lx >= 0.0f ? 1.0f : -1.0f; nly = 0.0f; pen = px + O_BALL_R; }
    else { nlx = 0.0f; nly = ly >= 0.0f ? 1.0f : -1.0f; pen = py + O_BALL_R; }
  }
  float nx = c * nlx - s * nly;
  float ny = s * nlx + c * nly;
  float pr = pen * O_W_ROBOT_BR, pb = pen * O_W_BALL_BR;
  b->x[i] = b->x[i] - nx * pr; b->y[i] = b->y[i] - ny * pr;
  b->bx = b->bx + nx * pb; b->by = b->by + ny * pb;
  float vn = (b->bvx - b->vx[i]) * nx + (b->bvy - b->vy[i]) * ny;
  if (vn < 0.0f) {
    float jr = vn * O_W_ROBOT_BR, jb = vn * O_W_BALL_BR;
    b->vx[i] = b->vx[i] + nx * jr; b->vy[i] = b->vy[i] + ny * jr;
    b->bvx = b->bvx - nx * jb; b->bvy = b->bvy - ny * jb;
  }
}

/* Disc of radius r against the field walls (envs/vss.py:449-518), folded into x,y >= 0. */
static void contact_walls(float* x, float* y, float* vx, float* vy, float r) {
  float sx = *x < 0.0f ? -1.0f : 1.0f, sy = *y < 0.0f ? -1.0f : 1.0f;
  float ax = fabsf(*x), ay = fabsf(*y);
  float avx = *vx * sx, avy = *vy * sy;
  if (ax <= O_FIELD_HX) {
    if (ay <= O_GOAL_HY) { /* near the goal post corner (0.75, 0.2) */
      float dx = ax - O_FIELD_HX, dy = ay - O_GOAL_HY;
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
    } else { /* facing an end wall x = 0.75 */
      float pen = ax + r - O_FIELD_HX;
      if (pen > 0.0f) { ax = ax - pen; if (avx > 0.0f) avx = 0.0f; }
    }
  } else {
    if (ay <= O_GOAL_HY) { /* inside the goal pocket: side faces y = +-0.2 */
      float pen = ay + r - O_GOAL_HY;
      if (pen > 0.0f) { ay = ay - pen; if (avy > 0.0f) avy = 0.0f; }
    } else { /* centre inside the end wall: shortest way out */
      float px = ax - O_FIELD_HX + r, py = ay - O_GOAL_HY + r;
      if (px < py) { ax = ax - px; if (avx > 0.0f) avx = 0.0f; }
      else { ay = ay - py; if (avy > 0.0f) avy = 0.0f; }
    }
  }
  { float pen = ay + r - O_FIELD_HY; if (pen > 0.0f) { ay = ay - pen; if (avy > 0.0f) avy = 0.0f; } }
  { float pen = ax + r - O_GOAL_BACK_X; if (pen > 0.0f) { ax = ax - pen; if (avx > 0.0f) avx = 0.0f; } }
  *x = ax * sx; *y = ay * sy; *vx = avx * sx; *vy = avy * sy;
}

static void physics_field(body_state* b, const float a[12]) {
  float tl[6], tr[6];
  for (int i = 0; i < 6; ++i) {
    /* DOF velocity targets a*42 rad/s (envs/vss.py:186) -> wheel rim speed */
    tl[i] = (a[2 * i] * O_WHEEL_RAD_S) * O_WHEEL_R;
    tr[i] = (a[2 * i + 1] * O_WHEEL_RAD_S) * O_WHEEL_R;
    heading(b, i);
  }
  for (int sub = 0; sub < O_NSUB; ++sub) {
    for (int i = 0; i < 6; ++i) { /* differential drive with traction-limited wheels */
      float c = b->c[i], s = b->s[i];
      float vf = c * b->vx[i] + s * b->vy[i];
      float vl = c * b->vy[i] - s * b->vx[i];
      float wl = vf - b->w[i] * O_HALF_TRACK;
      float wr = vf + b->w[i] * O_HALF_TRACK;
      wl = wl + clampf(tl[i] - wl, -O_DV, O_DV);
      wr = wr + clampf(tr[i] - wr, -O_DV, O_DV);
      vf = (wl + wr) * 0.5f;
      b->w[i] = (wr - wl) * O_INV_TRACK;
      vl = vl - clampf(vl, -O_DL, O_DL);
      b->vx[i] = c * vf - s * vl;
      b->vy[i] = s * vf + c * vl;
    }
    b->bvx = b->bvx * O_K_BALL;
    b->bvy = b->bvy * O_K_BALL;
    for (int i = 0; i < 6; ++i) {
      b->x[i] = b->x[i] + b->vx[i] * O_H;
      b->y[i] = b->y[i] + b->vy[i] * O_H;
      float sh, ch;
      oracle_sincosf(b->w[i] * O_HH, &sh, &ch);
      float qz = b->qz[i] * ch + b->qw[i] * sh;
      float qw = b->qw[i] * ch - b->qz[i] * sh;
      float k = 1.5f - 0.5f * (qz * qz + qw * qw); /* one Newton step of 1/|q| */
      b->qz[i] = qz * k;
      b->qw[i] = qw * k;
      heading(b, i);
    }
    b->bx = b->bx + b->bvx * O_H;
    b->by = b->by + b->bvy * O_H;
    for (int i = 0; i < 6; ++i)
      for (int j = i + 1; j < 6; ++j) contact_robot_robot(b, i, j);
    for (int i = 0; i < 6; ++i) contact_ball_robot(b, i);
    for (int i = 0; i < 6; ++i) contact_walls(&b->x[i], &b->y[i], &b->vx[i], &b->vy[i], O_ROBOT_R);
    contact_walls(&b->bx, &b->by, &b->bvx, &b->bvy, O_BALL_R);
  }
}

static void load_body(const float* st, int64_t n, int64_t f, body_state* b) {
  b->bx = CH(st, VSS_CH_BALL_X, n, f); b->by = CH(st, VSS_CH_BALL_Y, n, f);
  b->bvx = CH(st, VSS_CH_BALL_VX, n, f); b->bvy = CH(st, VSS_CH_BALL_VY, n, f);
  for (int i = 0; i < 6; ++i) {
    b->x[i] = CH(st, VSS_CH_RX + i, n, f); b->y[i] = CH(st, VSS_CH_RY + i, n, f);
    b->qz[i] = CH(st, VSS_CH_RQZ + i, n, f); b->qw[i] = CH(st, VSS_CH_RQW + i, n, f);
    b->vx[i] = CH(st, VSS_CH_RVX + i, n, f); b->vy[i] = CH(st, VSS_CH_RVY + i, n, f);
    b->w[i] = CH(st, VSS_CH_RW + i, n, f);
  }
}

static void store_body(float* st, int64_t n, int64_t f, const body_state* b) {
  CH(st, VSS_CH_BALL_X, n, f) = b->bx; CH(st, VSS_CH_BALL_Y, n, f) = b->by;
  CH(st, VSS_CH_BALL_VX, n, f) = b->bvx; CH(st, VSS_CH_BALL_VY, n, f) = b->bvy;
  for (int i = 0; i < 6; ++i) {
    CH(st, VSS_CH_RX + i, n, f) = b->x[i]; CH(st, VSS_CH_RY + i, n, f) = b->y[i];
    CH(st, VSS_CH_RQZ + i, n, f) = b->qz[i]; CH(st, VSS_CH_RQW + i, n, f) = b->qw[i];
    CH(st, VSS_CH_RVX + i, n, f) = b->vx[i]; CH(st, VSS_CH_RVY + i, n, f) = b->vy[i];
    CH(st, VSS_CH_RW + i, n, f) = b->w[i];
  }
}

int oracle_simulate(int64_t n, float* state, const float* actions) {
  if (n < 0 || !state || !actions) return VSS_E_ARG;
  for (int64_t f = 0; f < n; ++f) {
    body_state b;
    load_body(state, n, f, &b);
    physics_field(&b, actions + f * 12);
    store_body(state, n, f, &b);
  }
  return VSS_OK;
}

/* ------------------------------------------------------------------------------------------
 * Reward / done kernels (envs/vss.py:578-655), restated per field.
 * ---------------------------------------------------------------------------------------- */
/* compute_goal_rew, envs/vss.py:578-594: +1 ball in the right (yellow) goal, -1 left */
static int64_t goal_of(float bx, float by) {
  int is_goal = (fabsf(bx) > O_FIELD_HX) && (fabsf(by) < O_GOAL_HY);
  if (is_goal && bx > 0.0f) return 1;
  if (is_goal && bx < 0.0f) return -1;
  return 0;
}

/* compute_grad_rew potential, envs/vss.py:601-609; yellow_goal = (0.75, 0) (154-159) */
static float ball_potential(float bx, float by) {
  float lx = bx - (-O_FIELD_HX), ly = by - (-0.0f);
  float rx = bx - O_FIELD_HX, ry = by - 0.0f;
  return sqrtf(lx * lx + ly * ly) - sqrtf(rx * rx + ry * ry);
}

static float dist2d(float ax, float ay, float bx, float by) {
  float dx = ax - bx, dy = ay - by;
  return sqrtf(dx * dx + dy * dy);
}

void oracle_goal_rew(int64_t n, const float* ball, int64_t* goal) {
  for (int64_t f = 0; f < n; ++f) goal[f] = goal_of(ball[2 * f], ball[2 * f + 1]);
}

void oracle_grad_rew(int64_t n, const float* prev, const float* ball, float* grad) {
  for (int64_t f = 0; f < n; ++f)
    grad[f] = ball_potential(ball[2 * f], ball[2 * f + 1]) - ball_potential(prev[2 * f], prev[2 * f + 1]);
}

/* compute_move_rew, envs/vss.py:615-625: approach the ball (same sign for both teams) */
void oracle_move_rew(int64_t n, const float* prev_r, const float* r, const float* prev_b,
                     const float* b, float* move) {
  for (int64_t f = 0; f < n; ++f)
    for (int k = 0; k < 6; ++k) {
      float pd = dist2d(prev_r[f * 12 + 2 * k], prev_r[f * 12 + 2 * k + 1], prev_b[2 * f], prev_b[2 * f + 1]);
      float d = dist2d(r[f * 12 + 2 * k], r[f * 12 + 2 * k + 1], b[2 * f], b[2 * f + 1]);
      move[f * 6 + k] = pd - d;
    }
}

/* compute_vss_dones, envs/vss.py:634-655 */
void oracle_vss_dones(int64_t n, const float* ball, const int64_t* progress, int64_t max_len,
                      int64_t* reset) {
  for (int64_t f = 0; f < n; ++f) {
    int is_goal = (fabsf(ball[2 * f]) > O_FIELD_HX) && (fabsf(ball[2 * f + 1]) < O_GOAL_HY);
    int64_t r = is_goal ? 1 : 0;
    if (progress[f] >= max_len) r = 1;
    reset[f] = r;
  }
}

/* ------------------------------------------------------------------------------------------
 * Observations: compute_obs, envs/vss.py:530-575.  52 floats per agent: ball (4); own team
 * in rotation order starting with self (perms, envs/vss.py:173-175) x 9; opponents x 7.
 * Yellow agents see the field rotated by 180 deg (mirror_tensor, envs/vss.py:533-538,560).
 * cos/sin(yaw) are taken from the quaternion: cos = w^2 - z^2, sin = 2wz (the reference's
 * atan2 -> cos/sin of get_euler_xyz, equal within rounding; pinned by golden G1).
 * ---------------------------------------------------------------------------------------- */
static void robot_features(const float* st, int64_t n, int64_t f, const float* dof, int r,
                           float out[9]) {
  float qz = CH(st, VSS_CH_RQZ + r, n, f), qw = CH(st, VSS_CH_RQW + r, n, f);
  out[0] = CH(st, VSS_CH_RX + r, n, f);
  out[1] = CH(st, VSS_CH_RY + r, n, f);
  out[2] = CH(st, VSS_CH_RVX + r, n, f);
  out[3] = CH(st, VSS_CH_RVY + r, n, f);
  out[4] = qw * qw - qz * qz;
  out[5] = 2.0f * qw * qz;
  out[6] = CH(st, VSS_CH_RW + r, n, f);
  out[7] = dof[f * 12 + 2 * r];
  out[8] = dof[f * 12 + 2 * r + 1];
}

int oracle_compute_observations(int64_t n, const vss_state* st, float* obs, int32_t n_agents) {
  if (n < 0 || !st || !obs || !(n_agents == 1 || n_agents == 3 || n_agents == 6)) return VSS_E_ARG;
  const float* s = st->state;
  for (int64_t f = 0; f < n; ++f) {
    float ball[4] = {CH(s, 0, n, f), CH(s, 1, n, f), CH(s, 2, n, f), CH(s, 3, n, f)};
    float rob[6][9];
    for (int r = 0; r < 6; ++r) robot_features(s, n, f, st->dof_velocity_buf, r, rob[r]);
    for (int a = 0; a < n_agents; ++a) {
      int team = a / 3, idx = a % 3;
      float sgn = team == 0 ? 1.0f : -1.0f;
      float* o = obs + (f * n_agents + a) * 52;
      int j = 0;
      for (int q = 0; q < 4; ++q) o[j++] = team == 0 ? ball[q] : -ball[q];
      for (int k = 0; k < 3; ++k) {
        const float* rf = rob[team * 3 + (idx + k) % 3];
        for (int q = 0; q < 9; ++q) o[j++] = q < 6 ? rf[q] * sgn : rf[q];
      }
      for (int k = 0; k < 3; ++k) {
        const float* rf = rob[(1 - team) * 3 + k];
        for (int q = 0; q < 7; ++q) o[j++] = q < 6 ? rf[q] * sgn : rf[q];
      }
    }
  }
  return VSS_OK;
}

/* ------------------------------------------------------------------------------------------
 * reset_dones, envs/vss.py:267-333 (batch form: rejection rounds over the still-close fields
 * in ascending order, then angles, then ball velocities -- the reference's draw order).
 * ---------------------------------------------------------------------------------------- */
static int positions_too_close(const float pos[7][2]) {
  for (int i = 0; i < 7; ++i)
    for (int j = i + 1; j < 7; ++j)
      if (dist2d(pos[i][0], pos[i][1], pos[j][0], pos[j][1]) < O_MIN_DIST) return 1;
  return 0;
}

static int reset_fields(int64_t n, const vss_params* p, const vss_state* st, provider* pv,
                        const int64_t* ids, int64_t n_ids, uint32_t ext) {
  (void)p;
  if (n_ids == 0) return VSS_OK;
  float* s = st->state;
  float (*pos)[7][2] = (float (*)[7][2])malloc(sizeof(float) * 14 * (size_t)n_ids);
  uint8_t* close = (uint8_t*)malloc((size_t)n_ids);
  if (!pos || !close) { free(pos); free(close); return VSS_E_ARG; }
  const float scale_x = 1.5f - 0.14f, scale_y = 1.3f - 0.14f; /* field_scale envs/vss.py:142-147 */
  memset(close, 1, (size_t)n_ids);
  for (uint32_t round = 0;; ++round) {
    int any = 0;
    for (int64_t i = 0; i < n_ids; ++i) {
      if (!close[i]) continue;
      uint32_t f = (uint32_t)ids[i], ctr = st->rng_counter[ids[i]];
      for (int k = 0; k < 14; ++k) {
        float u = draw_uniform(pv, f, ctr, O_PURPOSE_POS | (ext >> 24), round, (uint32_t)k);
        pos[i][k / 2][k % 2] = (u - 0.5f) * (k % 2 == 0 ? scale_x : scale_y);
      }
    }
    for (int64_t i = 0; i < n_ids; ++i) {
      if (!close[i]) continue;
      close[i] = (uint8_t)positions_too_close(pos[i]);
      if (close[i] && round + 1 >= O_MAX_REJECT_ROUNDS) close[i] = 0; /* bounded */
      any |= close[i];
    }
    if (!any) break;
  }
  for (int64_t i = 0; i < n_ids; ++i) {
    int64_t f = ids[i];
    /* root_state[env_ids] = env_reset_root_state: zero velocities (envs/vss.py:272) */
    CH(s, VSS_CH_BALL_X, n, f) = pos[i][0][0];
    CH(s, VSS_CH_BALL_Y, n, f) = pos[i][0][1];
    for (int r = 0; r < 6; ++r) {
      CH(s, VSS_CH_RX + r, n, f) = pos[i][1 + r][0];
      CH(s, VSS_CH_RY + r, n, f) = pos[i][1 + r][1];
      CH(s, VSS_CH_RVX + r, n, f) = 0.0f;
      CH(s, VSS_CH_RVY + r, n, f) = 0.0f;
      CH(s, VSS_CH_RW + r, n, f) = 0.0f;
    }
  }
  /* rand_angles = torch_rand_float(-pi, pi, (n, 6)); quat_from_angle_axis (envs/vss.py:307-315) */
  for (int64_t i = 0; i < n_ids; ++i) {
    int64_t f = ids[i];
    uint32_t ctr = st->rng_counter[f];
    for (int r = 0; r < 6; ++r) {
      float u = draw_uniform(pv, (uint32_t)f, ctr, O_PURPOSE_ANG | (ext >> 24), 0, (uint32_t)r);
      float ang = O_TWO_PI * u + (-O_PI);
      float sh, ch;
      oracle_sincosf(ang * 0.5f, &sh, &ch);
      float nrm = sqrtf(sh * sh + ch * ch);
      CH(s, VSS_CH_RQZ + r, n, f) = sh / nrm;
      CH(s, VSS_CH_RQW + r, n, f) = ch / nrm;
    }
  }
  /* rand_ball_vel = (rand(n, 2) - 0.5) * 1 (envs/vss.py:318-327) */
  for (int64_t i = 0; i < n_ids; ++i) {
    int64_t f = ids[i];
    uint32_t ctr = st->rng_counter[f];
    for (int c = 0; c < 2; ++c) {
      float u = draw_uniform(pv, (uint32_t)f, ctr, O_PURPOSE_ANG | (ext >> 24), 0, (uint32_t)(6 + c));
      CH(s, VSS_CH_BALL_VX + c, n, f) = u - 0.5f;
    }
  }
  /* dof_velocity_buf[env_ids] *= 0.0 (envs/vss.py:333) */
  for (int64_t i = 0; i < n_ids; ++i)
    for (int k = 0; k < 12; ++k) st->dof_velocity_buf[ids[i] * 12 + k] *= 0.0f;
  free(pos);
  free(close);
  return VSS_OK;
}

static int64_t collect_resets(int64_t n, const int64_t* reset_buf, int64_t* ids) {
  int64_t m = 0;
  for (int64_t f = 0; f < n; ++f)
    if (reset_buf[f] != 0) ids[m++] = f;
  return m;
}

int oracle_reset_dones(int64_t n, const vss_params* p, const vss_state* st, oracle_draws* draws) {
  if (n < 0 || !p || !st) return VSS_E_ARG;
  provider pv = {p, draws};
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!ids) return VSS_E_ARG;
  int64_t m = collect_resets(n, st->reset_buf, ids);
  int rc = reset_fields(n, p, st, &pv, ids, m, O_EXTERNAL);
  /* an external reset consumes the field's counter so repeated calls draw afresh */
  for (int64_t i = 0; i < m; ++i) st->rng_counter[ids[i]] += 1u;
  free(ids);
  return rc;
}

/* ------------------------------------------------------------------------------------------
 * The step.  Ext VecTask.step: clamp (clipActions) → pre_physics_step → simulate →
 * post_physics_step → time_outs = (progress >= max_len - 1) & reset.
 * ---------------------------------------------------------------------------------------- */
int oracle_step(int64_t n, int32_t mode, const vss_params* p, const vss_state* st,
                const vss_step_io* io, oracle_draws* draws) {
  if (n < 0 || !p || !st || !io || mode < VSS_MODE_FULL || mode > VSS_MODE_DMA) return VSS_E_ARG;
  if (!st->state || !st->progress_buf || !st->reset_buf || !st->dof_velocity_buf || !st->rng_counter)
    return VSS_E_ARG;
  if (!io->actions || !io->obs || !io->terminal_obs || !io->rew || !io->time_outs || !io->progress_f)
    return VSS_E_ARG;
  if (mode != VSS_MODE_FULL && (!io->ou_buf || !io->reward_sum)) return VSS_E_ARG;
  if (mode == VSS_MODE_DMA && !io->dones_rep) return VSS_E_ARG;
  provider pv = {p, draws};
  float* s = st->state;
  const int R = mode == VSS_MODE_DMA ? 3 : 1;
  const int n_agents = mode == VSS_MODE_FULL ? 6 : (mode == VSS_MODE_DMA ? 3 : 1);
  float* acts = (float*)malloc(sizeof(float) * 12 * (size_t)(n > 0 ? n : 1));
  float* prev = (float*)malloc(sizeof(float) * 14 * (size_t)(n > 0 ? n : 1));
  float* rew = (float*)malloc(sizeof(float) * 24 * (size_t)(n > 0 ? n : 1));
  float* obs6 = (float*)malloc(sizeof(float) * 312 * (size_t)(n > 0 ? n : 1));
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!acts || !prev || !rew || !obs6 || !ids) {
    free(acts); free(prev); free(rew); free(obs6); free(ids);
    return VSS_E_ARG;
  }

  /* wrapper: action_buf = random_ou(action_buf); learner slots overwritten
   * (envs/wrappers.py:5-19,102-103,134-135,164-165) */
  if (mode == VSS_MODE_FULL) {
    memcpy(acts, io->actions, sizeof(float) * 12 * (size_t)n);
  } else {
    for (int64_t f = 0; f < n; ++f) {
      float z[12];
      draw_ou_noise(&pv, (uint32_t)f, st->rng_counter[f], z);
      float* ab = io->ou_buf + f * 12;
      for (int k = 0; k < 12; ++k) ab[k] = clampf((ab[k] - O_OU_THETA * ab[k]) + z[k], -1.0f, 1.0f);
      int nl = mode == VSS_MODE_SA ? 2 : 6;
      for (int k = 0; k < nl; ++k) ab[k] = io->actions[f * nl + k];
      memcpy(acts + f * 12, ab, sizeof(float) * 12);
    }
  }
  /* VecTask.step: actions = clamp(actions, -clip, clip) */
  for (int64_t i = 0; i < 12 * n; ++i) acts[i] = clampf(acts[i], -p->clip_actions, p->clip_actions);

  /* pre_physics_step, envs/vss.py:180-187 */
  for (int64_t f = 0; f < n; ++f) {
    if (st->reset_buf[f] != 0) st->progress_buf[f] = 0;
    memcpy(st->dof_velocity_buf + f * 12, acts + f * 12, sizeof(float) * 12);
  }
  /* prev positions (clone before refresh, envs/vss.py:219-220) */
  for (int64_t f = 0; f < n; ++f) {
    prev[f * 14 + 0] = CH(s, 0, n, f);
    prev[f * 14 + 1] = CH(s, 1, n, f);
    for (int r = 0; r < 6; ++r) {
      prev[f * 14 + 2 + 2 * r] = CH(s, VSS_CH_RX + r, n, f);
      prev[f * 14 + 3 + 2 * r] = CH(s, VSS_CH_RY + r, n, f);
    }
  }
  /* gym.simulate */
  oracle_simulate(n, s, st->dof_velocity_buf);

  /* post_physics_step, envs/vss.py:189-203 */
  for (int64_t f = 0; f < n; ++f) st->progress_buf[f] += 1;

  /* compute_rewards_and_dones, envs/vss.py:218-265 */
  for (int64_t f = 0; f < n; ++f) {
    float bx = CH(s, 0, n, f), by = CH(s, 1, n, f);
    float pbx = prev[f * 14], pby = prev[f * 14 + 1];
    float* rw = rew + f * 24;
    for (int k = 0; k < 24; ++k) rw[k] = 0.0f;
    int64_t g = goal_of(bx, by);
    float grad = ball_potential(bx, by) - ball_potential(pbx, pby);
    for (int a = 0; a < 6; ++a) {
      int team = a / 3;
      if (p->w_goal > 0.0f) rw[a * 4 + 0] = (float)(team == 0 ? g : -g) * p->w_goal;
      if (p->w_grad > 0.0f) rw[a * 4 + 1] = (team == 0 ? grad : -grad) * p->w_grad;
      if (p->w_move > 0.0f) {
        float pd = dist2d(prev[f * 14 + 2 + 2 * a], prev[f * 14 + 3 + 2 * a], pbx, pby);
        float d = dist2d(CH(s, VSS_CH_RX + a, n, f), CH(s, VSS_CH_RY + a, n, f), bx, by);
        rw[a * 4 + 2] = 0.0f + (pd - d) * p->w_move;
      }
      if (p->w_energy > 0.0f) {
        const float* dv = st->dof_velocity_buf + f * 12 + 2 * a;
        rw[a * 4 + 3] = 0.0f + (-((fabsf(dv[0]) + fabsf(dv[1])) / 2.0f)) * p->w_energy;
      }
    }
    int is_goal = (fabsf(bx) > O_FIELD_HX) && (fabsf(by) < O_GOAL_HY);
    st->reset_buf[f] = (is_goal || st->progress_buf[f] >= (int64_t)p->max_episode_length) ? 1 : 0;
  }

  /* terminal observation (envs/vss.py:195-196) and progress copy (198-200) */
  oracle_compute_observations(n, st, obs6, 6);
  for (int64_t f = 0; f < n; ++f) {
    for (int a = 0; a < n_agents; ++a)
      memcpy(io->terminal_obs + (f * n_agents + a) * 52, obs6 + (f * 6 + a) * 52, sizeof(float) * 52);
    for (int k = 0; k < R; ++k) io->progress_f[f * R + k] = (float)st->progress_buf[f];
  }

  /* reset_dones (envs/vss.py:202) */
  int64_t m = collect_resets(n, st->reset_buf, ids);
  reset_fields(n, p, st, &pv, ids, m, 0u);

  /* compute_observations again (envs/vss.py:203) */
  oracle_compute_observations(n, st, obs6, 6);
  for (int64_t f = 0; f < n; ++f)
    for (int a = 0; a < n_agents; ++a)
      memcpy(io->obs + (f * n_agents + a) * 52, obs6 + (f * 6 + a) * 52, sizeof(float) * 52);

  for (int64_t f = 0; f < n; ++f) {
    int64_t done = st->reset_buf[f];
    uint8_t to = (uint8_t)((st->progress_buf[f] >= (int64_t)p->max_episode_length - 1) && done != 0);
    for (int k = 0; k < R; ++k) io->time_outs[f * R + k] = to;
    const float* rw = rew + f * 24;
    if (mode == VSS_MODE_FULL) {
      memcpy(io->rew + f * 24, rw, sizeof(float) * 24);
      if (io->reward_sum) io->reward_sum[f] = ((rw[0] + rw[1]) + rw[2]) + rw[3];
    } else if (mode == VSS_MODE_SA) { /* rewards[:, 0, 0] (envs/wrappers.py:108) */
      for (int c = 0; c < 4; ++c) io->rew[f * 4 + c] = rw[c];
      io->reward_sum[f] = ((rw[0] + rw[1]) + rw[2]) + rw[3];
    } else if (mode == VSS_MODE_CMA) { /* rewards[:, 0, :].mean(1) (envs/wrappers.py:140) */
      float m4[4];
      for (int c = 0; c < 4; ++c) m4[c] = ((rw[c] + rw[4 + c]) + rw[8 + c]) / 3.0f;
      for (int c = 0; c < 4; ++c) io->rew[f * 4 + c] = m4[c];
      io->reward_sum[f] = ((m4[0] + m4[1]) + m4[2]) + m4[3];
    } else { /* DMA: rewards[:, 0].reshape(-1, 4) (envs/wrappers.py:173) */
      for (int a = 0; a < 3; ++a) {
        for (int c = 0; c < 4; ++c) io->rew[(f * 3 + a) * 4 + c] = rw[a * 4 + c];
        io->reward_sum[f * 3 + a] = ((rw[a * 4] + rw[a * 4 + 1]) + rw[a * 4 + 2]) + rw[a * 4 + 3];
        io->dones_rep[f * 3 + a] = done;
      }
    }
    /* wrapper: action_buf[env_ids] *= 0 for done fields (envs/wrappers.py:105-107) */
    if (mode != VSS_MODE_FULL && done)
      for (int k = 0; k < 12; ++k) io->ou_buf[f * 12 + k] *= 0.0f;
    st->rng_counter[f] += 1u;
  }
  free(acts); free(prev); free(rew); free(obs6); free(ids);
  return VSS_OK;
}
