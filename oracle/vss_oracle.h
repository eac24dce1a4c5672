/*
 * vss_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, float32, single thread) of the reference's VSS step, used as the
 * parity checker for the HIP path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product path (rsoccer-isaac-cleanrl_amd/) never does.
 *
 * It follows the reference phase by phase (VecTask.step → pre_physics_step → simulate →
 * post_physics_step, envs/vss.py:180-333) over host buffers with the same layout as the
 * device ABI in include/vss.h.  The physics (`oracle_simulate`) restates the build's own 2D
 * model: PhysX is closed and absent, so dynamics parity with the reference is
 * unpinned; everything around the physics is pinned against golden vectors generated from
 * the reference's own Python (tests/golden/).
 *
 * Random draws come either from the counter-based Philox stream the HIP kernel uses (draws ==
 * NULL) or, for pinning against the reference, from recorded torch draws replayed in the
 * order the reference consumed them (`oracle_draws`).
 */
#ifndef VSS_ORACLE_H
#define VSS_ORACLE_H

#include <stdint.h>
#include "../include/vss.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_draws {
  const float* uniforms;  /* every torch.rand output, in call order (reset_dones) */
  int64_t n_uniforms;
  int64_t uniform_pos;    /* cursor, advanced by the oracle */
  const float* normals;   /* every torch.normal output (already * 0.15), in call order */
  int64_t n_normals;
  int64_t normal_pos;
} oracle_draws;

int oracle_abi_version(void);

/* Full step in `mode` (VSS_MODE_*), same contract as vss_step(). */
int oracle_step(int64_t n, int32_t mode, const vss_params* p, const vss_state* st,
                const vss_step_io* io, oracle_draws* draws);

/* VSS.reset_dones over all fields with reset_buf != 0. */
int oracle_reset_dones(int64_t n, const vss_params* p, const vss_state* st,
                       oracle_draws* draws);

/* compute_obs for agents [0, n_agents). */
int oracle_compute_observations(int64_t n, const vss_state* st, float* obs, int32_t n_agents);

/* Physics only: advance every field by one control step with clamped actions (N,12)
 * (used as the fake `gym.simulate` hook when generating golden vectors). */
int oracle_simulate(int64_t n, float* state, const float* actions);

/* Individual reference kernels, restated (for golden-vector tests). */
void oracle_goal_rew(int64_t n, const float* ball_pos /*(n,2)*/, int64_t* goal /*(n)*/);
void oracle_grad_rew(int64_t n, const float* prev_ball /*(n,2)*/, const float* ball,
                     float* grad /*(n)*/);
void oracle_move_rew(int64_t n, const float* prev_robots /*(n,6,2)*/, const float* robots,
                     const float* prev_ball, const float* ball, float* move /*(n,6)*/);
void oracle_vss_dones(int64_t n, const float* ball_pos, const int64_t* progress,
                      int64_t max_episode_length, int64_t* reset);

/* Reference-independent helpers exposed for unit tests. */
void oracle_philox(uint32_t key0, uint32_t key1, const uint32_t ctr[4], uint32_t out[4]);
float oracle_logf(float x);
void oracle_sincosf(float x, float* s, float* c);

#ifdef __cplusplus
}
#endif

#endif
