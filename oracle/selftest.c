/* selftest.c — TEST INFRASTRUCTURE ONLY.  Drives the oracle through every mode (full, SA, CMA,
 * DMA), resets and edge sizes so it can run under AddressSanitizer + UndefinedBehaviorSanitizer
 * (make -C oracle check-asan).  Exit code 0 = no sanitizer report and invariants held. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vss_oracle.h"

static int run(int64_t n, int32_t mode, int steps) {
  const int R = mode == VSS_MODE_DMA ? 3 : 1;
  const int A = mode == VSS_MODE_FULL ? 6 : (mode == VSS_MODE_DMA ? 3 : 1);
  const int W = mode == VSS_MODE_FULL ? 12 : (mode == VSS_MODE_SA ? 2 : 6);
  float* state = calloc((size_t)(VSS_STATE_CHANNELS * n), sizeof(float));
  int64_t* progress = calloc((size_t)n, sizeof(int64_t));
  int64_t* reset = calloc((size_t)n, sizeof(int64_t));
  float* dof = calloc((size_t)(12 * n), sizeof(float));
  uint32_t* ctr = calloc((size_t)n, sizeof(uint32_t));
  float* actions = malloc(sizeof(float) * (size_t)(W * n));
  float* ou = calloc((size_t)(12 * n), sizeof(float));
  float* obs = malloc(sizeof(float) * (size_t)(52 * A * n));
  float* tobs = malloc(sizeof(float) * (size_t)(52 * A * n));
  float* rew = malloc(sizeof(float) * (size_t)(mode == VSS_MODE_FULL ? 24 * n : 4 * A * n));
  float* rsum = malloc(sizeof(float) * (size_t)(R * n));
  int64_t* dones = malloc(sizeof(int64_t) * (size_t)(3 * n));
  uint8_t* to = malloc((size_t)(R * n));
  float* pf = malloc(sizeof(float) * (size_t)(R * n));
  for (int64_t f = 0; f < n; ++f) {
    reset[f] = 1;
    for (int r = 0; r < 6; ++r) state[(VSS_CH_RQW + r) * n + f] = 1.0f;
  }
  vss_params p = {10.f, 2.f, 3.f, 0.5f, 1.f, 37, 99};
  vss_state st = {state, progress, reset, dof, ctr};
  vss_step_io io = {actions, ou, obs, tobs, rew, rsum, dones, to, pf};
  int bad = oracle_reset_dones(n, &p, &st, NULL);
  srand(7);
  for (int t = 0; t < steps && !bad; ++t) {
    for (int64_t i = 0; i < W * n; ++i) actions[i] = 2.6f * ((float)rand() / (float)RAND_MAX) - 1.3f;
    bad |= oracle_step(n, mode, &p, &st, &io, NULL);
    for (int64_t i = 0; i < VSS_STATE_CHANNELS * n && !bad; ++i) bad |= !isfinite(state[i]);
    for (int64_t i = 0; i < 52 * A * n && !bad; ++i) bad |= !isfinite(obs[i]) || !isfinite(tobs[i]);
    for (int64_t f = 0; f < n && !bad; ++f) bad |= progress[f] < 1 || progress[f] > p.max_episode_length;
    if (t % 50 == 17) {  /* external reset of every other field (play.py style) */
      for (int64_t f = 0; f < n; f += 2) reset[f] = 1;
      bad |= oracle_reset_dones(n, &p, &st, NULL);
    }
  }
  free(state); free(progress); free(reset); free(dof); free(ctr); free(actions); free(ou);
  free(obs); free(tobs); free(rew); free(rsum); free(dones); free(to); free(pf);
  return bad;
}

int main(void) {
  int bad = 0;
  const int64_t sizes[] = {1, 3, 64, 67};
  for (int m = VSS_MODE_FULL; m <= VSS_MODE_DMA; ++m)
    for (int s = 0; s < 4; ++s) bad |= run(sizes[s], m, 300);
  bad |= oracle_step(0, VSS_MODE_FULL, NULL, NULL, NULL, NULL) != VSS_E_ARG;
  printf(bad ? "oracle selftest FAILED\n" : "oracle selftest ok\n");
  return bad;
}
