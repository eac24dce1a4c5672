/*
 * vss_host_demo.c — the VSS C ABI (include/vss.h) driven from plain C, no Python, no torch.
 *
 * What a non-Python host (a C/C++ trainer, or the body of a cgo / JNI / N-API binding) does:
 * allocate the device buffers, reset every field, then one vss_step per control step on its own
 * stream.  Checks status codes, the argument refusal path and a few state invariants, and times
 * the steps with HIP events.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude examples/vss_host_demo.c \
 *       -Lrsoccer-isaac-cleanrl_amd/vss_amd -lvss_amd -L/opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/rsoccer-isaac-cleanrl_amd/vss_amd -o vss_host_demo
 *   ./vss_host_demo [fields=4096] [steps=200]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_runtime_api.h>

#include "vss.h"

#define HIP_OK(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return 2;                                                                        \
    }                                                                                  \
  } while (0)

#define VSS_OK_(call)                                                                  \
  do {                                                                                 \
    int rc_ = (call);                                                                  \
    if (rc_ != VSS_OK) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #call, vss_error_string(rc_)); \
      return 3;                                                                        \
    }                                                                                  \
  } while (0)

static float uniform(uint64_t* s) { /* xorshift64*, [-1, 1) */
  *s ^= *s >> 12; *s ^= *s << 25; *s ^= *s >> 27;
  return (float)((*s * 2685821657736338717ull) >> 40) / (float)(1ull << 24) * 2.0f - 1.0f;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
  const int steps = argc > 2 ? atoi(argv[2]) : 200;
  if (vss_abi_version() != VSS_ABI_VERSION) {
    fprintf(stderr, "ABI version %d, header %d\n", vss_abi_version(), VSS_ABI_VERSION);
    return 1;
  }
  const size_t ch = VSS_STATE_CHANNELS;
  float *state, *dof, *actions, *obs, *tobs, *rew, *progress_f;
  int64_t *progress, *reset;
  uint32_t* ctr;
  uint8_t* time_outs;
  HIP_OK(hipMalloc((void**)&state, ch * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&dof, 12 * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&actions, 12 * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&obs, 312 * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&tobs, 312 * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&rew, 24 * n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&progress_f, n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&progress, n * sizeof(int64_t)));
  HIP_OK(hipMalloc((void**)&reset, n * sizeof(int64_t)));
  HIP_OK(hipMalloc((void**)&ctr, n * sizeof(uint32_t)));
  HIP_OK(hipMalloc((void**)&time_outs, n));

  /* initial state: bodies at rest, unit quaternions; every field flagged for reset */
  float* h_state = (float*)calloc(ch * n, sizeof(float));
  int64_t* h_one = (int64_t*)malloc(n * sizeof(int64_t));
  for (int r = 0; r < 6; ++r)
    for (int64_t f = 0; f < n; ++f) h_state[(VSS_CH_RQW + r) * n + f] = 1.0f;
  for (int64_t f = 0; f < n; ++f) h_one[f] = 1;
  HIP_OK(hipMemcpy(state, h_state, ch * n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(reset, h_one, n * sizeof(int64_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemset(progress, 0, n * sizeof(int64_t)));
  HIP_OK(hipMemset(ctr, 0, n * sizeof(uint32_t)));
  HIP_OK(hipMemset(dof, 0, 12 * n * sizeof(float)));

  hipStream_t stream;
  HIP_OK(hipStreamCreate(&stream));
  vss_params p = {10.0f, 2.0f, 3.0f, 0.0f, 1.0f, 400, 1234};
  vss_state s = {state, progress, reset, dof, ctr};
  VSS_OK_(vss_reset_dones(stream, n, &p, &s));

  /* random actions U[-1, 1), one batch reused (the kernel reads it once per step) */
  float* h_act = (float*)malloc(12 * n * sizeof(float));
  uint64_t rng = 88172645463325252ull;
  for (int64_t i = 0; i < 12 * n; ++i) h_act[i] = uniform(&rng);
  HIP_OK(hipMemcpy(actions, h_act, 12 * n * sizeof(float), hipMemcpyHostToDevice));
  vss_step_io io = {actions, NULL, obs, tobs, rew, NULL, NULL, time_outs, progress_f};

  /* the refusal path: a misaligned observation pointer is VSS_E_ARG, nothing launched */
  vss_step_io bad = io;
  bad.obs = obs + 1;
  if (vss_step(stream, n, VSS_MODE_FULL, &p, &s, &bad) != VSS_E_ARG) {
    fprintf(stderr, "misaligned buffer was not refused\n");
    return 4;
  }

  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  VSS_OK_(vss_step(stream, n, VSS_MODE_FULL, &p, &s, &io)); /* warm-up */
  HIP_OK(hipEventRecord(e0, stream));
  for (int k = 0; k < steps; ++k) VSS_OK_(vss_step(stream, n, VSS_MODE_FULL, &p, &s, &io));
  HIP_OK(hipEventRecord(e1, stream));
  HIP_OK(hipStreamSynchronize(stream));
  float ms = 0.0f;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));

  /* invariants: finite, inside the walls, bookkeeping in range */
  float* h_obs = (float*)malloc(312 * n * sizeof(float));
  int64_t* h_prog = (int64_t*)malloc(n * sizeof(int64_t));
  int64_t* h_reset = (int64_t*)malloc(n * sizeof(int64_t));
  HIP_OK(hipMemcpy(h_state, state, ch * n * sizeof(float), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(h_obs, obs, 312 * n * sizeof(float), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(h_prog, progress, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(h_reset, reset, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  int64_t bad_values = 0, dones = 0;
  for (int64_t i = 0; i < 312 * n; ++i) bad_values += !isfinite(h_obs[i]);
  for (int64_t f = 0; f < n; ++f) {
    for (int b = 0; b < 7; ++b) {
      const float x = b == 0 ? h_state[VSS_CH_BALL_X * n + f] : h_state[(VSS_CH_RX + b - 1) * n + f];
      const float y = b == 0 ? h_state[VSS_CH_BALL_Y * n + f] : h_state[(VSS_CH_RY + b - 1) * n + f];
      bad_values += !(fabsf(x) < 0.86f && fabsf(y) < 0.66f);
    }
    bad_values += !(h_prog[f] >= 1 && h_prog[f] <= p.max_episode_length);
    bad_values += !(h_reset[f] == 0 || h_reset[f] == 1);
    dones += h_reset[f];
  }
  printf("{\"fields\": %lld, \"steps\": %d, \"us_per_step\": %.2f, \"env_steps_per_s\": %.4g, "
         "\"dones_last_step\": %lld, \"bad_values\": %lld, \"status\": \"%s\"}\n",
         (long long)n, steps, 1e3 * ms / steps, (double)n * steps / (ms * 1e-3), (long long)dones,
         (long long)bad_values, bad_values ? "FAIL" : "ok");
  return bad_values ? 5 : 0;
}
