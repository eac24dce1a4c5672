// Profiling-only: how v_mfma_f32_16x16x32_bf16 rounds its fp32 result (the x6 GEMMs' accumulation).
// Output element (0, 0) = C + sum over 32 k of A[0][k] B[k][0]; every case sets C and a few products whose
// exact sum is not an fp32 value, and prints the result next to what round-to-nearest-even, round toward
// zero and round toward -inf would give (computed on the host in double, then rounded).
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_rounding_probe tools/mfma_rounding_probe.hip && /tmp/mfma_rounding_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

// lane l holds A[row = l & 15][k = 8 (l >> 4) .. + 7] and B[k = 8 (l >> 4) .. + 7][col = l & 15]; the
// accumulator lane l holds D[rows 4 (l >> 4) .. + 3][col l & 15]
__global__ void mfma_case(const uint16_t* a, const uint16_t* b, const float* c, float* d) {
  const int l = threadIdx.x;
  u16x8 av, bv;
  for (int e = 0; e < 8; ++e) {
    av[e] = a[(l & 15) * 32 + 8 * (l >> 4) + e];
    bv[e] = b[(8 * (l >> 4) + e) * 16 + (l & 15)];
  }
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c[(4 * (l >> 4) + r) * 16 + (l & 15)];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

static uint16_t bf(float x) {  // exact for the values used here
  uint32_t u;
  memcpy(&u, &x, 4);
  return (uint16_t)(u >> 16);
}

static float round_mode(double v, int mode) {  // 0 RNE, 1 toward zero, 2 toward -inf
  float f = (float)v;  // RNE
  if (mode == 0) return f;
  if ((double)f == v) return f;
  float lo = (double)f < v ? f : nextafterf(f, -INFINITY);
  float hi = (double)f < v ? nextafterf(f, INFINITY) : f;
  if (mode == 1) return v > 0 ? lo : hi;
  return lo;
}

int main() {
  struct Case {
    const char* name;
    float c;
    int n;
    float p[4];  // products p[i] = a[i] * 1.0
  } cases[] = {
      {"1 + 0.75 ulp", 1.0f, 1, {0x1.8p-24f}},
      {"1 + 0.25 ulp", 1.0f, 1, {0x1.0p-25f}},
      {"1 - 0.75 ulp(below 1)", 1.0f, 1, {-0x1.8p-25f}},
      {"-1 - 0.75 ulp", -1.0f, 1, {-0x1.8p-24f}},
      {"-1 - 0.25 ulp", -1.0f, 1, {-0x1.0p-25f}},
      {"1 + 0.5 ulp (tie)", 1.0f, 1, {0x1.0p-24f}},
      {"1 + 1.5 ulp (tie)", 1.0f, 1, {0x1.8p-23f}},
      {"1 + 4 x 0.3 ulp (sum 1.2 ulp)", 1.0f, 4, {0x1.34p-25f, 0x1.34p-25f, 0x1.34p-25f, 0x1.34p-25f}},
      {"0 + 1 + 0.75 ulp (C = 0)", 0.0f, 2, {1.0f, 0x1.8p-24f}},
      {"0 + 1 - 0.75 ulp(below) (C = 0)", 0.0f, 2, {1.0f, -0x1.8p-25f}},
      {"0 - 1 - 0.75 ulp (C = 0)", 0.0f, 2, {-1.0f, -0x1.8p-24f}},
      {"C = +0.75 ulp, product 1", 0x1.8p-24f, 1, {1.0f}},
      {"C = -0.375 ulp, product 1", -0x1.8p-25f, 1, {1.0f}},
      {"C = +0.375 ulp, product 1", 0x1.8p-25f, 1, {1.0f}},
      {"C = -0.75 ulp, product -1", -0x1.8p-24f, 1, {-1.0f}},
      {"C = +2^-30, product 1", 0x1.0p-30f, 1, {1.0f}},
      {"C = -2^-30, product 1", -0x1.0p-30f, 1, {1.0f}},
      {"1 + 2^-30 (far below)", 1.0f, 1, {0x1.0p-30f}},
      {"1 - 2^-30 (far below)", 1.0f, 1, {-0x1.0p-30f}},
      {"-1 + 2^-30 (far below)", -1.0f, 1, {0x1.0p-30f}},
      {"-1 - 2^-30 (far below)", -1.0f, 1, {-0x1.0p-30f}},
  };
  uint16_t *da, *db;
  float *dc, *dd;
  hipMalloc(&da, 16 * 32 * 2);
  hipMalloc(&db, 32 * 16 * 2);
  hipMalloc(&dc, 256 * 4);
  hipMalloc(&dd, 256 * 4);
  for (const Case& cs : cases) {
    uint16_t a[16 * 32] = {0}, b[32 * 16] = {0};
    float c[256] = {0}, d[256];
    double exact = cs.c;
    for (int i = 0; i < cs.n; ++i) {
      a[0 * 32 + 5 * i + 1] = bf(cs.p[i]);  // spread over k groups
      b[(5 * i + 1) * 16 + 0] = bf(1.0f);
      const uint32_t back = (uint32_t)bf(cs.p[i]) << 16;
      float pv;
      memcpy(&pv, &back, 4);
      exact += (double)pv;
    }
    c[0] = cs.c;
    hipMemcpy(da, a, sizeof a, hipMemcpyHostToDevice);
    hipMemcpy(db, b, sizeof b, hipMemcpyHostToDevice);
    hipMemcpy(dc, c, sizeof c, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_case, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
    hipMemcpy(d, dd, sizeof d, hipMemcpyDeviceToHost);
    const float rne = round_mode(exact, 0), rtz = round_mode(exact, 1), rdn = round_mode(exact, 2);
    printf("{\"case\": \"%s\", \"exact\": %.12g, \"mfma\": \"%a\", \"rne\": \"%a\", \"toward_zero\": \"%a\", "
           "\"toward_minus_inf\": \"%a\", \"matches\": \"%s%s%s\"}\n",
           cs.name, exact, d[0], rne, rtz, rdn, d[0] == rne ? "rne " : "", d[0] == rtz ? "rtz " : "",
           d[0] == rdn ? "rdn" : "");
  }
  return 0;
}
