/*
 * vss.h — C ABI of the MI355X-native VSS (IEEE Very Small Size, 3v3) match step.
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json `north_star`:
 * the reference's `VSS.step` (envs/vss.py:180-333 + the Ext IsaacGymEnvs VecTask.step that
 * drives it, + PhysX `gym.simulate`) and the SA/CMA/DMA wrapper packing
 * (envs/wrappers.py:5-19,89-180).  The Python classes in
 * `rsoccer-isaac-cleanrl_amd/envs/{vss,wrappers}.py` bind these entry points with ctypes.
 *
 * Conventions:
 *   - every buffer is a caller-owned DEVICE allocation (torch tensors); the library allocates
 *     nothing and keeps no hidden state besides what is passed in;
 *   - all work is enqueued on `stream` (a hipStream_t passed as void*); no host synchronisation;
 *   - return value 0 = ok, otherwise a VSS_E_* code (vss_error_string() describes it);
 *   - runtime parameters (reward weights, episode length, clip, seed) are passed per call.
 *
 * Field state layout (struct-of-arrays, fp32, `state[channel * n_fields + field]`), chosen so
 * the reference's tensor views (envs/vss.py:112-132) are plain strided views of one buffer:
 *   VSS_CH_BALL_X..VSS_CH_BALL_VY             ball x, y, vx, vy
 *   VSS_CH_RX + r, VSS_CH_RY + r               robot r position      (r = team*3 + robot)
 *   VSS_CH_RQX..VSS_CH_RQW + r                 robot r quaternion x,y,z,w (x,y unused: planar)
 *   VSS_CH_RVX + r, VSS_CH_RVY + r             robot r linear velocity
 *   VSS_CH_RW + r                              robot r yaw rate
 */
#ifndef VSS_AMD_VSS_H
#define VSS_AMD_VSS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSS_ABI_VERSION 2

#define VSS_NUM_TEAMS 2          /* envs/vss.py:24 */
#define VSS_NUM_ROBOTS 3         /* envs/vss.py:25 */
#define VSS_NUM_AGENTS 6
#define VSS_NUM_OBS 52           /* envs/vss.yaml:4, layout envs/vss.py:530-575 */
#define VSS_NUM_ACTIONS 2        /* envs/vss.yaml:5 (left wheel, right wheel) */
#define VSS_NUM_REW 4            /* goal, grad, move, energy: envs/vss.py:90-92 */

/* state channels */
#define VSS_CH_BALL_X 0
#define VSS_CH_BALL_Y 1
#define VSS_CH_BALL_VX 2
#define VSS_CH_BALL_VY 3
#define VSS_CH_RX 4
#define VSS_CH_RY 10
#define VSS_CH_RQX 16
#define VSS_CH_RQY 22
#define VSS_CH_RQZ 28
#define VSS_CH_RQW 34
#define VSS_CH_RVX 40
#define VSS_CH_RVY 46
#define VSS_CH_RW 52
#define VSS_STATE_CHANNELS 58

/* which wrapper the step is fused with (envs/wrappers.py:43-48) */
#define VSS_MODE_FULL 0  /* raw VSS.step: actions (N,2,3,2), obs (N,2,3,52), rew (N,2,3,4) */
#define VSS_MODE_SA 1    /* SingleAgent: learner = blue robot 0 (envs/wrappers.py:89-115)   */
#define VSS_MODE_CMA 2   /* CMA: learner = blue team, one 6-vector (envs/wrappers.py:118-148) */
#define VSS_MODE_DMA 3   /* DMA: learner = blue robots 0..2, one row each (wrappers.py:151-180) */

/* Alignment (checked; VSS_E_ARG otherwise): observation, reward, dof_velocity, OU and FULL /
 * rollout action buffers 16 B (float4 access); SA/CMA/DMA action buffers 8 B; int64 buffers 8 B;
 * packed MLP weights 16 B.  Allocator (hipMalloc / torch) pointers always qualify; a view at an
 * odd element offset may not. */

/* error codes */
#define VSS_OK 0
#define VSS_E_ARG 1      /* null or misaligned pointer / bad size / bad mode */
#define VSS_E_LAUNCH 2   /* kernel launch failed (hipGetLastError) */

typedef struct vss_params {
  float w_goal;              /* rew_weights.goal   envs/vss.yaml:9,  envs/vss.py:44 */
  float w_grad;              /* rew_weights.grad   envs/vss.yaml:10 */
  float w_move;              /* rew_weights.move   envs/vss.yaml:11 */
  float w_energy;            /* rew_weights.energy envs/vss.yaml:12 */
  float clip_actions;        /* env.clipActions    envs/vss.yaml:7 (Ext VecTask clamp) */
  int32_t max_episode_length;/* env.maxEpisodeLength envs/vss.yaml:6 */
  uint64_t seed;             /* Philox key for reset sampling and OU noise */
} vss_params;

typedef struct vss_state {
  float* state;              /* [VSS_STATE_CHANNELS][n_fields] fp32 SoA (see above)       */
  int64_t* progress_buf;     /* [n_fields]   envs/vss.py:95                               */
  int64_t* reset_buf;        /* [n_fields]   envs/vss.py:93                               */
  float* dof_velocity_buf;   /* [n_fields][2][3][2] last clamped actions, envs/vss.py:137  */
  uint32_t* rng_counter;     /* [n_fields]   per-field Philox step counter                */
} vss_state;

/*
 * Per-step inputs/outputs.  Shapes by mode (N = n_fields, R = 3 for DMA else 1):
 *   actions      FULL (N,2,3,2) | SA (N,2) | CMA (N,6) | DMA (3N,2)             read
 *   ou_buf       wrapper action buffer (N,2,3,2); SA/CMA/DMA only                 read+write
 *   obs          FULL (N,2,3,52) | SA/CMA (N,52) | DMA (3N,52)                     write
 *   terminal_obs same shape as obs (pre-reset observation)                        write
 *   rew          FULL (N,2,3,4) | SA/CMA (N,4) | DMA (3N,4)                        write
 *   reward_sum   SA/CMA (N,) | DMA (3N,) = rews.sum(-1); may be NULL in FULL       write
 *   dones_rep    DMA only: (3N,) int64 = dones.repeat_interleave(3); else NULL     write
 *   time_outs    (R*N,) uint8 (torch.bool)                                          write
 *   progress_f   (R*N,) fp32 = progress_buf.float() before the reset              write
 */
typedef struct vss_step_io {
  const float* actions;
  float* ou_buf;
  float* obs;
  float* terminal_obs;
  float* rew;
  float* reward_sum;
  int64_t* dones_rep;
  uint8_t* time_outs;
  float* progress_f;
} vss_step_io;

/*
 * Open-loop rollout buffers for vss_rollout (K = n_steps, N = n_fields), step-major:
 *   actions      (K,N,2,3,2) fp32                                                   read
 *   obs          (K,N,2,3,52), terminal_obs (K,N,2,3,52), rew (K,N,2,3,4) fp32      write
 *   dones        (K,N) int64 = reset_buf after each step                            write
 *   time_outs    (K,N) uint8, progress_f (K,N) fp32                                 write
 */
typedef struct vss_rollout_io {
  const float* actions;
  float* obs;
  float* terminal_obs;
  float* rew;
  int64_t* dones;
  uint8_t* time_outs;
  float* progress_f;
} vss_rollout_io;

/*
 * Recorded random draws for the parity entries vss_step_replay / vss_reset_dones_replay: the
 * reference's own torch draws, so the product kernels can be run against golden fixtures made by
 * the reference (tests/golden/) instead of the Philox stream.  Per field f, row
 * uniforms[f * uniform_stride ...] holds the draws the reference's reset_dones consumed for f in
 * this call, in its order (envs/vss.py:267-333):
 *   14 per rejection round r at [14 r, 14 r + 14): f's (7, 2) row of
 *      torch.rand((len(close_ids), 7, 2)) (ball, then robots blue 0-2, yellow 0-2; x, y)
 *      in the rounds where f was still too close (envs/vss.py:281-299);
 *   then, after the R rounds f used, [14 R, 14 R + 6): f's row of torch_rand_float(-pi, pi,
 *      (n, 6)) (robot yaws, envs/vss.py:307-312) and [14 R + 6, 14 R + 8): f's row of
 *      torch.rand((n, 2)) (ball velocity, envs/vss.py:318-325).
 * Rows of fields that do not reset are not read.  uniform_stride >= 22; a row holds
 * (uniform_stride - 8) / 14 rounds (capped at 64, the product's bound).
 * normals (SA/CMA/DMA; may be NULL in FULL): (n_fields, 12), the step's
 * torch.normal(0, 0.15, (N, 2, 3, 2)) of random_ou (envs/wrappers.py:5-19), already scaled.
 */
typedef struct vss_replay_draws {
  const float* uniforms;
  int64_t uniform_stride;
  const float* normals;
} vss_replay_draws;

/* ABI version (VSS_ABI_VERSION). */
int vss_abi_version(void);

/* The build's source stamp: 16 hex digits of sha256 over the library's sources (csrc/Makefile
 * STAMPED).  The Python loader recomputes it from the tree and refuses a stale library. */
const char* vss_source_hash(void);

/* Human-readable text for a VSS_E_* code. */
const char* vss_error_string(int code);

/*
 * One control step of every field.  Replaces, for mode FULL, Ext VecTask.step →
 * VSS.pre_physics_step (envs/vss.py:180-187) → gym.simulate → VSS.post_physics_step
 * (envs/vss.py:189-203) → time_outs; for SA/CMA/DMA additionally the wrapper's
 * random_ou + learner overwrite + slicing (envs/wrappers.py:101-115, 133-148, 163-180).
 */
int vss_step(void* stream, int64_t n_fields, int32_t mode, const vss_params* params,
             const vss_state* st, const vss_step_io* io);

/*
 * Parity entry: vss_step with the reset and OU draws taken from `draws` (recorded reference
 * draws, see vss_replay_draws) instead of the Philox stream.  The same kernel template as
 * vss_step (REPLAY instantiation); everything but the draw source is shared.  Test use only.
 */
int vss_step_replay(void* stream, int64_t n_fields, int32_t mode, const vss_params* params,
                    const vss_state* st, const vss_step_io* io, const vss_replay_draws* draws);

/*
 * K consecutive FULL-mode steps in one launch for a pre-supplied action sequence (random-action
 * benchmarks, scripted / OU opponents, evaluation): bit-identical to K vss_step(FULL) calls — the
 * same reference semantics per step (envs/vss.py:180-333) — with the field state kept on chip
 * between steps.  State buffers (st) are updated as after the K-th step.
 */
int vss_rollout(void* stream, int64_t n_fields, int32_t n_steps, const vss_params* params,
                const vss_state* st, const vss_rollout_io* io);

/*
 * Re-sample every field whose reset_buf != 0 (VSS.reset_dones, envs/vss.py:267-333);
 * callable externally after `reset_buf[:] = 1` (play.py:132-133).  Does not touch
 * reset_buf / progress_buf and does not compute observations (same as the reference).
 */
int vss_reset_dones(void* stream, int64_t n_fields, const vss_params* params,
                    const vss_state* st);

/* Parity entry: vss_reset_dones with recorded reference draws (e.g. the construction-time
 * reset, envs/vss.py:72); normals unused.  Test use only. */
int vss_reset_dones_replay(void* stream, int64_t n_fields, const vss_params* params,
                           const vss_state* st, const vss_replay_draws* draws);

/*
 * compute_obs (envs/vss.py:205-216, 530-575) for agents [0, n_agents): n_agents = 6 writes
 * (N,2,3,52), 3 writes the blue team (N,3,52), 1 writes blue robot 0 (N,52).
 */
int vss_compute_observations(void* stream, int64_t n_fields, const vss_state* st,
                             float* obs, int32_t n_agents);

/* ---------------------------------------------------------------------------------------------
 * Fused rollout policy: the reference Agent's actor and critic MLPs
 * (ppo_continuous_action_isaacgym.py:127-164, 52 -> 256 -> 512 -> 512 -> 256 -> n_out, tanh)
 * on the fp32 matrix cores, activations kept in registers across the five layers.
 * ------------------------------------------------------------------------------------------- */

/* floats needed for one network's packed weights (n_out = 1 critic, 2 or 6 actor); -1 if bad */
int64_t vss_mlp_packed_size(int32_t n_out);

/*
 * Repack one network (torch nn.Linear layout: weights[i] is (out, in) row-major, biases[i] (out))
 * into the kernel's lane order.  Call once per parameter update.
 */
int vss_mlp_pack(void* stream, int32_t n_out, const float* const* weights, const float* const* biases,
                 float* packed);

/*
 * Agent.get_action_and_value (ppo…:157-164) on `rows` observations (rows, 52):
 * mean = actor(obs); action = action_in if given, else mean + exp(logstd) * N(0,1) (Philox on
 * (seed, counter, row)); log-prob and entropy summed over the n_act dims (torch Normal
 * formulas); value = critic(obs).  With actor_packed == NULL only the critic runs
 * (Agent.get_value, ppo…:154-155).  Any output pointer may be NULL.
 */
int vss_policy_forward(void* stream, int64_t rows, int32_t n_act, const float* obs,
                       const float* actor_packed, const float* logstd, const float* critic_packed,
                       uint64_t seed, uint64_t counter, const float* action_in, float* action_out,
                       float* logprob_out, float* entropy_out, float* value_out, float* mean_out);

/*
 * vss_policy_forward with an optional row mask for the critic-only form (actor_packed == NULL):
 * only rows with row_mask[row] != 0 (e.g. the step's dones) are evaluated and written.  Used
 * for the terminal-observation values of the fields that reset (ppo…:272): for every other field
 * the terminal observation equals the next observation, whose value the next step computes.
 */
int vss_value_forward_masked(void* stream, int64_t rows, int32_t n_act, const float* obs,
                             const float* actor_packed, const float* logstd, const float* critic_packed,
                             uint64_t seed, uint64_t counter, const float* action_in, float* action_out,
                             float* logprob_out, float* entropy_out, float* value_out, float* mean_out,
                             const int64_t* row_mask);

/*
 * The actor tail of Agent.get_action_and_value (ppo_continuous_action_isaacgym.py:157-164) from
 * actor means computed elsewhere (the rollout's GEMM-chain path, vss_amd/policy.py): per row,
 * action = mean + exp(logstd) z with z from the same Philox stream (seed, counter, row) as
 * vss_policy_forward (or action_in when given), log-prob and entropy summed over the n_act dims.
 * mean / action_in / action_out (rows, n_act), logprob_out / entropy_out (rows,); outputs may be NULL.
 */
int vss_policy_sample(void* stream, int64_t rows, int32_t n_act, const float* mean, const float* logstd, uint64_t seed,
                      uint64_t counter, const float* action_in, float* action_out, float* logprob_out,
                      float* entropy_out);

/* ---------------------------------------------------------------------------------------------
 * PPO-update helper: the backward of a hidden layer's tanh
 * (ppo_continuous_action_isaacgym.py:104-111, autograd of nn.Tanh + nn.Linear's bias) in one pass:
 *   grad_in = grad_out * (1 - y^2)             (rows, cols) row-major, y = tanh output
 *   bias_partial[c][j] = sum of grad_in[r][j] over the rows r of part c
 * with vss_tanh_grad_chunks(rows, cols) parts (fixed row sets, -1 for a bad size); the bias
 * gradient is the sum of bias_partial over its parts (caller-side, deterministic).  cols in {64, 128, 256, 512, 1024};
 * every pointer 16-B aligned.  Replaces torch's tanh_backward + the bias-gradient reduction.
 * ------------------------------------------------------------------------------------------- */
int64_t vss_tanh_grad_chunks(int64_t rows, int32_t cols);
int vss_tanh_grad_bias(void* stream, int64_t rows, int32_t cols, const float* grad_out, const float* y,
                       float* grad_in, float* bias_partial);

/*
 * The forward of a hidden layer (nn.Linear then nn.Tanh, ppo…:104-111; in the update:
 * ppo…:331 → Agent.get_action_and_value) in one launch on the fp32 matrix cores:
 * y = tanh(x W^T + b) with x (rows, k_in), W (n_out, k_in) (nn.Linear's layout), both row-major,
 * y (rows, n_out).  k_in % 4 == 0, n_out % 128 == 0; x, W, y 16-B aligned.  Replaces torch's
 * addmm + tanh (the activation is written once instead of written, read and written again).
 */
int vss_linear_tanh(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                    const float* bias, float* y);

/*
 * vss_linear_tanh for the LAST hidden layer with the output layer folded in (ppo…:104-111: Linear(512,
 * 256), Tanh, Linear(256, k_out)): y = tanh(x W^T + b) as vss_linear_tanh, and
 *   out_part[s][r][a] = sum over the 64 columns c of slice s (s = 0..3) of y[r][c] w_out[a][c]
 * so the output layer is out = sum_s out_part[s] + b_out without a second read of y.  n_out = 256,
 * rows % 256 == 0, k_in % 64 == 0, k_out in {1, 2, 6}; w_out (k_out, 256) row-major; out_part
 * (4, rows, k_out).  VSS_E_ARG for other shapes (the caller uses vss_linear_tanh + a GEMM then).
 */
int vss_linear_tanh_out(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                        const float* bias, float* y, int32_t k_out, const float* w_out, float* out_part);

/*
 * The backward through a layer and the tanh below it (autograd of nn.Linear → nn.Tanh,
 * ppo…:104-111, in loss.backward() at ppo…:357) in one launch on the fp32 matrix cores:
 *   grad_in = (grad_next W_next) * (1 - y^2),   bias_partial[c][j] = sum of grad_in[r][j] over part c
 * grad_next (rows, k_next) = the pre-activation gradient of the layer above, w_next_t (n_out, k_next)
 * = that layer's weight TRANSPOSED (row-major), y (rows, n_out) = this layer's tanh output,
 * grad_in (rows, n_out) = this layer's pre-activation gradient.  The bias gradient is the sum over
 * the vss_linear_tanh_backward_chunks(rows, k_next, n_out) parts (fixed, deterministic; -1 for a bad
 * shape).  k_next % 4 == 0, n_out % 128 == 0; every pointer 16-B aligned.  Replaces torch's dX GEMM +
 * vss_tanh_grad_bias (the gradient is written once instead of written, read and written again).
 */
int64_t vss_linear_tanh_backward_chunks(int64_t rows, int32_t k_next, int32_t n_out);
int vss_linear_tanh_backward(void* stream, int64_t rows, int32_t k_next, int32_t n_out, const float* grad_next,
                             const float* w_next_t, const float* y, float* grad_in, float* bias_partial);

/* The Agent's output layer backward in one streaming pass (ppo_continuous_action_isaacgym.py:104-111
 * under loss.backward(), :357): for the output nn.Linear (k_out = 1, 2 or 6 columns, g_out and its
 * weight zero-padded by the caller to k_pad = 4 or 8 columns / rows) over a tanh layer of width n
 * (n in {128, 256, 512, 1024}):
 *   grad_in = (g_out W_out) * (1 - y^2)        the tanh layer's pre-activation gradient (rows, n)
 *   bias_partial (chunks, n)                   column-sum parts of grad_in (its bias gradient)
 *   wgrad_partial (chunks, k_pad, n)           parts of g_out^T y, the output layer's weight gradient
 * g_out (rows, k_pad), w_out_t (n, k_pad) = the padded weight TRANSPOSED, y (rows, n) = the tanh
 * output (the output layer's input); chunks = vss_output_backward_chunks(rows, k_pad, n) (-1 for a
 * bad shape), summed in a fixed order by the caller.  Every pointer 16-B aligned.  Replaces the
 * output layer's dX GEMM + tanh_backward + bias reduction and its dW GEMM (two reads of y -> one).
 */
int64_t vss_output_backward_chunks(int64_t rows, int32_t k_pad, int32_t n);
int vss_output_backward(void* stream, int64_t rows, int32_t k_pad, int32_t n, const float* g_out, const float* w_out_t,
                        const float* y, float* grad_in, float* bias_partial, float* wgrad_partial);

/* vss_output_backward_direct: the same pass for the update's minibatch without autograd
 * (vss_amd/minibatch.py direct_minibatch): g_out (rows, k_out) as vss_ppo_loss_direct
 * writes it and w_out (k_out, n) as nn.Linear holds it -- no padded copies; k_out in {1, 2, 3, 4, 6, 8},
 * n in {128, 256, 512, 1024}.  bias_partial (chunks, n), wgrad_partial (chunks, k_out, n) with chunks =
 * vss_output_backward_direct_chunks(rows, k_out, n) <= 256 (-1 for a bad shape), few enough for one
 * vss_sum_parts launch.  y, grad_in and the partials 16-B aligned; g_out, w_out 4-B aligned.
 */
int64_t vss_output_backward_direct_chunks(int64_t rows, int32_t k_out, int32_t n);
int vss_output_backward_direct(void* stream, int64_t rows, int32_t k_out, int32_t n, const float* g_out,
                               const float* w_out, const float* y, float* grad_in, float* bias_partial,
                               float* wgrad_partial);

/* ---------------------------------------------------------------------------------------------
 * The update's hidden-layer GEMMs in fp32 arithmetic on the bf16 matrix cores (csrc/vss_gemm_x6.hip;
 * ppo_continuous_action_isaacgym.py:104-111 under the update's forward ppo…:331 and loss.backward()
 * ppo…:357).  Every fp32 operand is split exactly into three bf16 parts (hi + mid + lo) and each
 * product is the six partial products above 2^-23 |a||b|, accumulated in fp32: the error is that of
 * an fp32 GEMM (tests/test_gemm_x6.py).  Exact shapes only (the update's minibatches); VSS_E_ARG
 * otherwise, and the caller uses the fp32-MFMA entries above.
 *
 * vss_linear_tanh_bf16x6 / _out_bf16x6 / vss_linear_tanh_backward_bf16x6: the same contracts as
 * vss_linear_tanh / vss_linear_tanh_out / vss_linear_tanh_backward with rows % 256 == 0,
 * n_out % 128 == 0, k % 64 == 0 (k_in resp. k_next); the backward's bias gradient is the sum over the
 * vss_linear_tanh_backward_chunks_bf16x6 parts.  w_split: caller-owned scratch of 3 * n_out * k
 * uint16 (16-B aligned) that the call fills with the weight's bf16 planes before its GEMM reads them.
 *
 * w (resp. w_next_t) == NULL: w_split already holds the weight's planes, written by
 * vss_weight_planes_bf16x6 for this (n_out, k) since the weight last changed (no split launch).
 *
 * vss_weight_planes_bf16x6: the planes of `count` (1..16) weights in ONE launch, into the w_split
 * buffers the GEMM entries above then take with a NULL weight: job q is an (n[q], k[q]) operand
 * (n % 128 == 0, n <= 4096, k % 64 == 0), stored row-major as w[q] (n, k) when transpose[q] == 0, or
 * as its transpose (k, n) when transpose[q] == 1 (the backward's W_next^T straight from nn.Linear's
 * weight, no transposed copy).  Host arrays of `count` entries; w_split 16-B aligned, w 16-B
 * aligned when not transposed.  Replaces one split launch per GEMM and the backward's transposes.
 *
 * vss_weight_grad_bf16x6: a Linear layer's weight gradient (autograd of nn.Linear, ppo…:357)
 *   partial[s][o][i] = sum over the rows r of part s of grad[r][o] x[r][i]
 * grad (rows, n_out) = the layer's output gradient, x (rows, k_in) = its input; dW = the sum over the
 * vss_weight_grad_chunks_bf16x6(rows, n_out, k_in) parts (-1 for a bad shape).  rows % 64 == 0,
 * n_out % 256 == 0, k_in % 128 == 0; every pointer 16-B aligned.  Replaces hipBLASLt's split-K
 * grad^T x GEMM.
 *
 * vss_first_weight_grad_bf16x6: the same for the Agent's FIRST layer (nn.Linear(obs, 256),
 * ppo_continuous_action_isaacgym.py:131,142; its weight gradient under loss.backward(), ppo…:352),
 * whose input x (rows, k_in) is the observation: n_out == 256, k_in <= 64 and k_in % 4 == 0 (52 for
 * every VSS wrapper), rows % 64 == 0; grad and x 16-B aligned.  partial (parts, 256, k_in), parts =
 * vss_first_weight_grad_chunks_bf16x6(rows, n_out, k_in) (-1 for a bad shape).  Replaces hipBLASLt's
 * batched grad^T x + torch.sum (the split-K dW of the first layer).
 *
 * vss_first_layer_bf16x6: the Agent's FIRST layer forward, y = tanh(x W^T + b) (nn.Linear(obs, 256) +
 * nn.Tanh, ppo…:131,142) with x (rows, k_in) the observations, w (256, k_in) nn.Linear's weight,
 * bias (256,), y (rows, 256): n_out == 256, 0 < k_in <= 64, k_in % 4 == 0, any rows >= 0; x and y
 * 16-B aligned.  The same split products as above (k zero-padded to 64); tanh as the other epilogues.
 * Replaces the fp32-MFMA first_layer_kernel (vss_linear_tanh) on the update and rollout paths.
 * ------------------------------------------------------------------------------------------- */
int vss_linear_tanh_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                           const float* bias, float* y, uint16_t* w_split);
int vss_linear_tanh_out_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x,
                               const float* w, const float* bias, float* y, int32_t k_out, const float* w_out,
                               float* out_part, uint16_t* w_split);
int64_t vss_linear_tanh_backward_chunks_bf16x6(int64_t rows, int32_t k_next, int32_t n_out);
int vss_linear_tanh_backward_bf16x6(void* stream, int64_t rows, int32_t k_next, int32_t n_out, const float* grad_next,
                                    const float* w_next_t, const float* y, float* grad_in, float* bias_partial,
                                    uint16_t* w_split);
/* vss_linear_tanh_loss_bf16x6: the last hidden layer, the output layer, the minibatch's PPO loss terms and
 * the output layer's backward in ONE x6 launch (direct_minibatch): y = tanh(x W^T + b) stays in the
 * accumulators, out = y w_out^T + b_out, each row's loss terms and gradient g_out as vss_ppo_loss_direct
 * forms them (role 0: the actor's policy terms, k_out in {1, 2}, advantages normalised from adv_part as
 * there; role 1: the critic's value terms, k_out == 1), and grad_in (rows_pad, 256) = (g_out w_out)
 * (1 - y^2) -- the hidden layer's pre-activation gradient, written instead of y.  Rows >= rows are
 * padding: zero gradient, no loss term.  Per block b of vss_linear_tanh_loss_blocks_bf16x6(rows_pad, k_in,
 * n_out) (-1 for a bad shape): part_cs[b] (256,) its column sums of grad_in (the hidden bias gradient),
 * part_dwo[b] (k_out, 256) its g_out^T y (the output weight gradient), part_stats[b] (32,) its loss sums
 * (csrc/vss_loss_row.h kBlockStats) for vss_ppo_loss_fused_finish.  n_out == 256, rows_pad % 256 == 0,
 * k_in % 64 == 0; w_split the weight's bf16 planes (vss_weight_planes_bf16x6), x / grad_in 16-B aligned.
 * Replaces vss_linear_tanh_out_bf16x6 + vss_ppo_loss_direct's row pass + vss_output_backward_direct. */
int64_t vss_linear_tanh_loss_blocks_bf16x6(int64_t rows, int32_t k_in, int32_t n_out);
int vss_linear_tanh_loss_bf16x6(void* stream, int32_t role, int64_t rows_pad, int64_t rows, int32_t k_in, int32_t n_out,
                                const float* x, const float* bias, int32_t k_out, const float* w_out, const float* b_out,
                                const float* action, const float* logprob_old, const float* adv, const double* adv_part,
                                int32_t adv_nparts, double adv_count, const float* logstd, const float* returns,
                                const float* values_old, float clip_coef, float clip_lo, float clip_hi, float vf_coef,
                                int32_t clip_vloss, float* grad_in, float* part_cs, float* part_dwo, float* part_stats,
                                const uint16_t* w_split);
int vss_weight_planes_bf16x6(void* stream, int32_t count, const float* const* w, const int32_t* n, const int32_t* k,
                             const int32_t* transpose, uint16_t* const* w_split);
int64_t vss_weight_grad_chunks_bf16x6(int64_t rows, int32_t n_out, int32_t k_in);
int vss_weight_grad_bf16x6(void* stream, int64_t rows, int32_t n_out, int32_t k_in, const float* grad, const float* x,
                           float* partial);
int vss_first_layer_bf16x6(void* stream, int64_t rows, int32_t k_in, int32_t n_out, const float* x, const float* w,
                           const float* bias, float* y);
int64_t vss_first_weight_grad_chunks_bf16x6(int64_t rows, int32_t n_out, int32_t k_in);
int vss_first_weight_grad_bf16x6(void* stream, int64_t rows, int32_t n_out, int32_t k_in, const float* grad,
                                 const float* x, float* partial);

/* ---------------------------------------------------------------------------------------------
 * The clipped PPO loss of one update minibatch and its gradients (SURVEY §8 A13;
 * ppo_continuous_action_isaacgym.py:314-349: Normal(mean, exp(logstd)).log_prob(action).sum(1), the
 * ratio to the rollout's log-prob, the clipped surrogate, the (optionally clipped) value loss, the
 * entropy, loss = pg_loss - ent_coef entropy_loss + vf_coef v_loss, and old_approx_kl / approx_kl /
 * clipfrac), in two launches.  Replaces torch's loss expressions and their autograd (~100 kernels).
 *   mean, action (rows_pad, n_act); value (rows_pad,) the critic output; logstd (n_act,);
 *   logprob_old, adv, returns, values_old (rows,) the minibatch's stored rows (adv already normalised);
 *   clip_lo / clip_hi: 1 - clip_coef and 1 + clip_coef as fp32 (the clamp bounds);
 *   grad_mean (rows_pad, n_act), grad_value (rows_pad,), grad_logstd (n_act,): d loss / d input, with
 *     torch's conventions at the kinks (maximum splits a tie in half, clamp passes [lo, hi]); rows
 *     [rows, rows_pad) (padding copies the loss does not see) get zero;
 *   loss_out[1] = loss; stats_out[6] = pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac;
 *   partial: scratch of vss_ppo_loss_scratch_floats(rows_pad, n_act) floats (-1 for a bad size),
 *     reduced in a fixed order (deterministic).
 * n_act in {1, 2, 3, 4, 6, 8}; every pointer 4-B aligned.
 * ------------------------------------------------------------------------------------------- */
int64_t vss_ppo_loss_scratch_floats(int64_t rows_pad, int32_t n_act);
int vss_ppo_loss(void* stream, int64_t rows, int64_t rows_pad, int32_t n_act, const float* mean, const float* logstd,
                 const float* value, const float* action, const float* logprob_old, const float* adv,
                 const float* returns, const float* values_old, float clip_coef, float clip_lo, float clip_hi,
                 float ent_coef, float vf_coef, int32_t clip_vloss, float* grad_mean, float* grad_value,
                 float* grad_logstd, float* loss_out, float* stats_out, float* partial);

/* vss_ppo_loss_direct: the same loss for the update's minibatch without autograd
 * (vss_amd/minibatch.py direct_minibatch), from what the networks' last launches leave:
 *   mean_parts (mean_nparts, rows_pad, n_act) + mean_bias (n_act,): the actor's output as the parts of
 *     vss_linear_tanh_out_bf16x6's out_part (summed in order, then the bias); value_parts
 *     (value_nparts, rows_pad) + value_bias (1,) the critic's;
 *   adv (rows,) RAW advantages, normalised in the kernel when adv_part != NULL: adv_part (adv_nparts, 2)
 *     fp64 (sum, sum of squares) parts over adv_count values (vss_minibatch_gather's, or their all-reduced
 *     sum), (a - mean) / (std + 1e-8) with mean = s / n, std = sqrt(max((q - n mean^2) / (n - 1), 0)) in
 *     fp64 (ppo…:325-326, normalize_advantages' data-parallel formula); adv_part NULL: adv as given;
 *   grad_mean_bias (n_act,), grad_value_bias (1,): the output layers' bias gradients (column sums of
 *     grad_mean / grad_value, fixed order), written like grad_logstd;
 * the other arguments as vss_ppo_loss; partial: vss_ppo_loss_direct_scratch_floats(rows_pad, n_act).
 *
 * vss_minibatch_gather: one update minibatch's rows (ppo…:310-317) in one launch: for r < rows_pad,
 *   i = inds[r < mb ? r : (r - mb) % mb] (the padding rows repeat the minibatch), obs[r] = b_obs[i]
 *   (obs_w floats), act[r] = b_act[i] (act_w floats); for r < mb, logp / adv / ret / val[r] = b_*[i];
 *   adv_part (vss_minibatch_gather_parts(mb), 2) fp64 (sum, sum of squares) parts of the gathered
 *   advantages (fixed order).  An index outside [0, batch) gathers NaN.  inds int64 (mb,).
 * vss_adv_part_sum: out[2] = the nparts parts summed in order (for the data-parallel all-reduce).
 */
int64_t vss_ppo_loss_direct_scratch_floats(int64_t rows_pad, int32_t n_act);
int vss_ppo_loss_direct(void* stream, int64_t rows, int64_t rows_pad, int32_t n_act, const float* mean_parts,
                        int32_t mean_nparts, const float* mean_bias, const float* value_parts, int32_t value_nparts,
                        const float* value_bias, const float* logstd, const float* action, const float* logprob_old,
                        const float* adv, const double* adv_part, int32_t adv_nparts, double adv_count,
                        const float* returns, const float* values_old, float clip_coef, float clip_lo, float clip_hi,
                        float ent_coef, float vf_coef, int32_t clip_vloss, float* grad_mean, float* grad_value,
                        float* grad_logstd, float* grad_mean_bias, float* grad_value_bias, float* loss_out,
                        float* stats_out, float* partial);
/* vss_ppo_loss_fused_finish: vss_linear_tanh_loss_bf16x6's per-block loss sums of the actor (actor_blocks)
 * and the critic (critic_blocks) -> loss_out[1], stats_out[6], grad_logstd, grad_mean_bias (n_act,) and
 * grad_value_bias (1,) as vss_ppo_loss_direct writes them; n_act in {1, 2}. */
int vss_ppo_loss_fused_finish(void* stream, int64_t rows, int32_t n_act, int64_t actor_blocks, const float* actor_stats,
                              int64_t critic_blocks, const float* critic_stats, const float* logstd, float ent_coef,
                              float vf_coef, float* grad_logstd, float* grad_mean_bias, float* grad_value_bias,
                              float* loss_out, float* stats_out);
/* vss_randperm: the epoch's minibatch permutation (ppo…:309, torch.randperm(batch)): out (n,) int64 a
 * uniformly random permutation of [0, n) determined by seed[0] (one int64 on the device, drawn from the
 * update's generator), 0 < n < 2^31.  scratch: vss_randperm_scratch_bytes(n) bytes (-1 for a bad n),
 * 256-B aligned.  Each index gets 32 random bits (splitmix64 of seed and index); a radix sort on them
 * (4 passes, hipcub) orders the indices, and every run of tied bits is then shuffled (Fisher-Yates from a
 * second stream), so the permutation is uniform.  vss_randperm_bits: the same with key_bits (1..32) random
 * bits per index -- fewer bits force ties (the tie pass's test entry); vss_randperm = key_bits 32. */
int64_t vss_randperm_scratch_bytes(int64_t n);
int vss_randperm(void* stream, int64_t n, const int64_t* seed, int64_t* out, void* scratch, int64_t scratch_bytes);
int vss_randperm_bits(void* stream, int64_t n, int32_t key_bits, const int64_t* seed, int64_t* out, void* scratch,
                      int64_t scratch_bytes);
int64_t vss_minibatch_gather_parts(int64_t mb);
int vss_minibatch_gather(void* stream, int64_t mb, int64_t rows_pad, int64_t batch, const int64_t* inds, int64_t obs_w,
                         int64_t act_w, const float* b_obs, const float* b_act, const float* b_logp, const float* b_adv,
                         const float* b_ret, const float* b_val, float* obs, float* act, float* logp, float* adv,
                         float* ret, float* val, double* adv_part);
int vss_adv_part_sum(void* stream, int32_t nparts, const double* part, double* out);

/* ---------------------------------------------------------------------------------------------
 * The update's gradient bookkeeping on flat buffers (csrc/vss_optim.hip; vss_amd/flat.py
 * FlatGrads / FlatAdam).  Replaces, per minibatch, nn.utils.clip_grad_norm_ (ppo…:353)
 * and optim.Adam(eps=1e-5).step() (ppo…:166,354) -- torch's per-tensor norm chain and multi-tensor
 * Adam -- with two launches, and the split GEMMs' torch.sum reductions with one launch per backward.
 *
 * vss_grad_sq_partials: partial[b] = sum of grad[i]^2 over block b's chunk, b < count =
 *   vss_grad_sq_partials_count(n) (<= 1024; -1 for n <= 0); fixed order (deterministic).
 * vss_adam_step_clipped: norm = sqrt(sum of the nparts partials); with max_norm >= 0 the gradients are
 *   scaled in place by min(1, max_norm / (norm + 1e-6)) (clip_grad_norm_: max_norm 0 zeroes them, as
 *   torch's does), with max_norm < 0 they are left alone (no clip requested); then Adam's step `step`
 *   (>= 1, the count after this step) with torch's fused-Adam arithmetic: m = b1 m + (1 - b1) g,
 *   v = b2 v + (1 - b2) g^2, p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps).
 *   norm_out (1 float, may be NULL) receives the pre-clip norm.  All buffers n fp32 elements.
 * vss_sum_parts: `count` (1..32) jobs; job q: dst[r * dst_ld + c] = sum over s = 0 .. parts - 1 of
 *   src[s * part_stride + r * src_ld + c], r < rows, c < cols, in a fixed order (parts s = w + 4 (u + 8 i)
 *   into running sum (w, u), then those sums in a fixed tree: deterministic).  Host arrays of count
 *   entries; device buffers; src parts must not overlap dst.
 * ------------------------------------------------------------------------------------------- */
int64_t vss_grad_sq_partials_count(int64_t n);
int vss_grad_sq_partials(void* stream, int64_t n, const float* grad, float* partial);
int vss_adam_step_clipped(void* stream, int64_t n, int32_t nparts, const float* partial, float max_norm, float lr,
                          float beta1, float beta2, float eps, int64_t step, float* grad, float* param, float* exp_avg,
                          float* exp_avg_sq, float* norm_out);
int vss_sum_parts(void* stream, int32_t count, const float* const* src, float* const* dst, const int64_t* parts,
                  const int64_t* part_stride, const int64_t* rows, const int64_t* cols, const int64_t* src_ld,
                  const int64_t* dst_ld);

/* ---------------------------------------------------------------------------------------------
 * Episode statistics: RecordEpisodeStatisticsTorch.step (envs/wrappers.py:66-87)
 * for `rows` learner rows in one launch, in the reference's order:
 *   ep_returns += rews; ep_lengths += 1; returned_returns = ep_returns; returned_lengths =
 *   ep_lengths; return_sum = ((r0 + r1) + r2) + r3 of returned_returns; then
 *   ep_returns *= 1 - dones; ep_lengths *= 1 - dones.
 * rews, ep_returns, returned_returns: (rows, 4) fp32, 16-B aligned; ep_lengths,
 * returned_lengths: (rows,) int32; dones: (rows,) int64; return_sum: (rows,) fp32.
 * ------------------------------------------------------------------------------------------- */
int vss_episode_stats(void* stream, int64_t rows, const float* rews, const int64_t* dones, float* ep_returns,
                      int32_t* ep_lengths, float* returned_returns, int32_t* returned_lengths, float* return_sum);

#ifdef __cplusplus
}
#endif

#endif /* VSS_AMD_VSS_H */
