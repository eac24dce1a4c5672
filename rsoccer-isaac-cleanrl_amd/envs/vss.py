"""Drop-in `VSS` vectorised 3v3 soccer task backed by the MI355X HIP match step.

Public surface = the reference's `envs/vss.py` class VSS (+ the Ext IsaacGymEnvs VecTask base
it inherits), so the reference's wrappers, PPO loop and `play.py` run unchanged against it:

  * ctor `VSS(cfg, rl_device, sim_device, graphics_device_id, headless,
    virtual_screen_capture, force_render)` (envs/vss.py:32-41) with the `cfg` keys of
    envs/vss.yaml;
  * `step(actions (N,2,3,2))` -> `(obs_dict, rew_buf (N,2,3,4), reset_buf (N,) int64, extras)`
    with extras `terminal_observation`, `progress_buffer`, `time_outs` (envs/vss.py:189-203 and
    Ext VecTask.step);
  * `reset()`, `reset_dones()` (envs/vss.py:267-333, callable after `reset_buf[:] = 1`,
    play.py:132-133), `compute_observations()`;
  * attributes `num_envs` / `num_environments`, `num_obs`, `num_actions`, `device`, `cfg`,
    `reset_buf`, `progress_buf`, `dof_velocity_buf`, `obs_buf`, `rew_buf`, mutable reward weights
    `w_goal / w_grad / w_move / w_energy`, observation/action spaces (2,3,52)/(2,3,2), and the
    state views `ball_pos, ball_vel, robots_pos, robots_vel, robots_quats, robots_ang_vel`
    (envs/vss.py:112-132) — writable strided views of the SoA state the kernel reads.

What differs by design: physics is the build's 2D model instead of PhysX; the
returned `obs_dict['obs']`, `rew_buf`, `reset_buf` and `extras[...]` are persistent buffers
overwritten by the next step (the reference returns clones for two of them; its train loop and
wrappers consume them before the next step either way); random draws come from a per-field
Philox stream keyed by `seed` instead of torch's generator.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from vss_amd import _native as N

from ._gym import Box

NUM_TEAMS = 2
NUM_ROBOTS = 3
BLUE_TEAM, YELLOW_TEAM = 0, 1


def default_cfg(num_envs: int = 4095) -> dict:
    """The task configuration (same keys and values as envs/vss.yaml)."""
    import yaml

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "vss.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["env"]["numEnvs"] = num_envs
    return cfg


class VSS:
    """Vectorised VSS fields on one GPU; one kernel launch per `step`."""

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id=0, headless=True,
                 virtual_screen_capture=False, force_render=False):
        env = cfg["env"]
        self.cfg = cfg
        self.num_fields = int(env["numEnvs"])
        self.max_episode_length = int(env["maxEpisodeLength"])
        self.w_goal = float(env["rew_weights"]["goal"])
        self.w_grad = float(env["rew_weights"]["grad"])
        self.w_move = float(env["rew_weights"]["move"])
        self.w_energy = float(env["rew_weights"]["energy"])
        self.robot_max_wheel_rad_s = 42.0
        self.min_robot_placement_dist = 0.07
        self.field_width, self.field_height = 1.5, 1.3
        self.goal_width, self.goal_height = 0.1, 0.4
        self.num_environments = self.num_fields
        self.num_observations = int(env["numObservations"])
        self.num_actions = int(env["numActions"])
        self.num_states = int(env.get("numStates", 0))
        self.clip_actions = float(env.get("clipActions", math.inf))
        self.clip_obs = float(env.get("clipObservations", math.inf))
        if self.num_observations != 52 or self.num_actions != 2:
            raise ValueError("VSS has 52 observations and 2 actions per robot (envs/vss.yaml:4-5)")
        if self.num_fields < 1:
            raise ValueError("numEnvs must be >= 1")
        self.device = N.require_device(sim_device)
        self.rl_device = torch.device(rl_device)
        self.graphics_device_id = graphics_device_id
        self.headless = headless
        self.viewer = None
        self.seed = int(env["seed"]) if "seed" in env else int(
            torch.randint(0, 2**62, (1,), dtype=torch.int64).item())

        self.obs_space = Box(-np.inf, np.inf, (NUM_TEAMS, NUM_ROBOTS, self.num_observations))
        self.state_space = Box(-np.inf, np.inf, (NUM_TEAMS, NUM_ROBOTS, self.num_states))
        self.act_space = Box(-1, 1, (NUM_TEAMS, NUM_ROBOTS, self.num_actions))

        self.allocate_buffers()
        self._acquire_tensors()
        self.obs_dict = {}
        self.extras = {}
        self.reset_dones()
        self.compute_observations()

    # ------------------------------------------------------------------------------ buffers
    def allocate_buffers(self):
        n, dev = self.num_fields, self.device
        self.state = torch.zeros((N.STATE_CHANNELS, n), device=dev, dtype=torch.float32)
        self.state[N.CH_RQW:N.CH_RQW + 6] = 1.0
        self.obs_buf = torch.zeros((n, NUM_TEAMS, NUM_ROBOTS, self.num_observations), device=dev)
        self.terminal_obs_buf = torch.zeros_like(self.obs_buf)
        self.states_buf = torch.zeros_like(self.obs_buf)
        self.rew_buf = torch.zeros((n, NUM_TEAMS, NUM_ROBOTS, 4), device=dev)
        self.reset_buf = torch.ones(n, device=dev, dtype=torch.long)
        self.timeout_buf = torch.zeros(n, device=dev, dtype=torch.bool)
        self.progress_buf = torch.zeros(n, device=dev, dtype=torch.long)
        self.progress_f_buf = torch.zeros(n, device=dev, dtype=torch.float32)
        self.randomize_buf = torch.zeros(n, device=dev, dtype=torch.long)
        self.dof_velocity_buf = torch.zeros((n, NUM_TEAMS, NUM_ROBOTS, 2), device=dev)
        self.rng_counter = torch.zeros(n, device=dev, dtype=torch.int32)  # uint32 bits

    def _acquire_tensors(self):
        """Reference-compatible views (envs/vss.py:112-132) over the SoA state."""
        n, s = self.num_fields, self.state
        self.ball_pos = s[N.CH_BALL_X:N.CH_BALL_X + 2].t()
        self.ball_vel = s[N.CH_BALL_VX:N.CH_BALL_VX + 2].t()
        robots = (n, NUM_TEAMS, NUM_ROBOTS)
        rstride = (1, NUM_ROBOTS * n, n)
        self.robots_pos = s.as_strided(robots + (2,), rstride + (6 * n,), N.CH_RX * n)
        self.robots_quats = s.as_strided(robots + (4,), rstride + (6 * n,), N.CH_RQX * n)
        self.robots_vel = s.as_strided(robots + (2,), rstride + (6 * n,), N.CH_RVX * n)
        self.robots_ang_vel = s.as_strided(robots + (1,), rstride + (1,), N.CH_RW * n)
        self.z_axis = torch.tensor([0.0, 0.0, 1.0], device=self.device)
        self.yellow_goal = torch.tensor([self.field_width / 2, 0.0], device=self.device)
        self.permutations = torch.tensor([[0, 1, 2], [1, 2, 0], [2, 0, 1]], device=self.device)

    def _c_params(self) -> N.VssParams:
        return N.VssParams(self.w_goal, self.w_grad, self.w_move, self.w_energy, self.clip_actions,
                           self.max_episode_length, self.seed & 0xFFFFFFFFFFFFFFFF)

    def _c_state(self) -> N.VssState:
        return N.VssState(self.state.data_ptr(), self.progress_buf.data_ptr(), self.reset_buf.data_ptr(),
                          self.dof_velocity_buf.data_ptr(), self.rng_counter.data_ptr())

    # ------------------------------------------------------------------------------ spaces
    @property
    def num_envs(self):
        return self.num_environments

    @property
    def num_obs(self):
        return self.num_observations

    @property
    def observation_space(self):
        return self.obs_space

    @property
    def action_space(self):
        return self.act_space

    # ------------------------------------------------------------------------------ the step
    def _check_buffer(self, name: str, t, numel: int, dtype: torch.dtype, required: bool = True):
        """A caller buffer the kernel writes: right size, dtype, device, contiguous (the kernel
        trusts its pointers, so a short buffer would be an out-of-bounds device write)."""
        if t is None:
            if required:
                raise ValueError(f"{name} is required")
            return
        if t.numel() != numel or t.dtype != dtype or t.device != self.device or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dtype} tensor of {numel} elements on {self.device}, "
                             f"got {tuple(t.shape)} {t.dtype} on {t.device}")

    def native_step(self, mode: int, actions: torch.Tensor, io: dict) -> None:
        """One fused step in `mode` (FULL / SA / CMA / DMA) writing into the tensors of `io`.

        Buffers are checked here (size, dtype, device, contiguity); the kernel itself is one
        launch on the current stream with no host synchronisation."""
        n = self.num_fields
        if mode not in (N.MODE_FULL, N.MODE_SA, N.MODE_CMA, N.MODE_DMA):
            raise ValueError(f"unknown mode {mode}")
        rows = {N.MODE_FULL: n, N.MODE_SA: n, N.MODE_CMA: n, N.MODE_DMA: 3 * n}[mode]   # output rows
        width = {N.MODE_FULL: 12, N.MODE_SA: 2, N.MODE_CMA: 6, N.MODE_DMA: 2}[mode]
        agents = {N.MODE_FULL: 6, N.MODE_SA: 1, N.MODE_CMA: 1, N.MODE_DMA: 3}[mode]     # obs rows per field
        if actions.numel() != rows * width:
            raise ValueError(f"actions must have {rows * width} elements, got {tuple(actions.shape)}")
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        full = mode == N.MODE_FULL
        r = 1 if full else rows  # time_outs / progress rows: per field, or per agent row for DMA
        self._check_buffer("io['obs']", io.get("obs"), n * agents * 52, torch.float32)
        self._check_buffer("io['terminal_obs']", io.get("terminal_obs"), n * agents * 52, torch.float32)
        self._check_buffer("io['rew']", io.get("rew"), n * 24 if full else rows * 4, torch.float32)
        self._check_buffer("io['reward_sum']", io.get("reward_sum"), rows, torch.float32, required=not full)
        self._check_buffer("io['ou_buf']", io.get("ou_buf"), n * 12, torch.float32, required=not full)
        self._check_buffer("io['dones_rep']", io.get("dones_rep"), rows, torch.long, required=mode == N.MODE_DMA)
        self._check_buffer("io['time_outs']", io.get("time_outs"), n if full else r, torch.bool)
        self._check_buffer("io['progress_f']", io.get("progress_f"), n if full else r, torch.float32)
        cio = N.VssStepIO(actions.data_ptr(), N.ptr(io.get("ou_buf")), N.ptr(io["obs"]),
                          N.ptr(io["terminal_obs"]), N.ptr(io["rew"]), N.ptr(io.get("reward_sum")),
                          N.ptr(io.get("dones_rep")), N.ptr(io["time_outs"]), N.ptr(io["progress_f"]))
        prm, st = self._c_params(), self._c_state()
        rc = N.load().vss_step(N.stream_of(self.device), n, mode, N.ctypes.byref(prm), N.ctypes.byref(st),
                               N.ctypes.byref(cio))
        N.check(rc, "vss_step")

    def step(self, actions: torch.Tensor):
        """Ext VecTask.step + VSS.pre/post_physics_step for every field (one HIP launch)."""
        self.native_step(N.MODE_FULL, actions, dict(
            obs=self.obs_buf, terminal_obs=self.terminal_obs_buf, rew=self.rew_buf, reward_sum=None,
            time_outs=self.timeout_buf, progress_f=self.progress_f_buf))
        self.extras["terminal_observation"] = self.terminal_obs_buf
        self.extras["progress_buffer"] = self.progress_f_buf
        self.extras["time_outs"] = self.timeout_buf
        self.obs_dict["obs"] = self._clipped(self.obs_buf)
        return self.obs_dict, self.rew_buf, self.reset_buf, self.extras

    def rollout(self, actions: torch.Tensor, out: dict | None = None) -> dict:
        """K FULL-mode steps of a pre-supplied action sequence `actions` (K, N, 2, 3, 2) in ONE
        launch (vss_rollout): identical to K `step()` calls, returning per-step tensors
        obs / terminal_observation (K,N,2,3,52), rew (K,N,2,3,4), dones (K,N) int64,
        time_outs (K,N) bool, progress_buffer (K,N).  For open-loop rollouts (scripted or OU
        opponents, random-action benchmarks); the env state ends as after the K-th step."""
        K = int(actions.shape[0])
        n = self.num_fields
        if actions.numel() != K * n * 12:
            raise ValueError(f"actions must be (K, {n}, 2, 3, 2), got {tuple(actions.shape)}")
        actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if out is not None:
            for k, (numel, dt) in dict(obs=(K * n * 312, torch.float32), terminal_observation=(K * n * 312, torch.float32),
                                       rew=(K * n * 24, torch.float32), dones=(K * n, torch.long),
                                       time_outs=(K * n, torch.bool), progress_buffer=(K * n, torch.float32)).items():
                self._check_buffer(f"out['{k}']", out.get(k), numel, dt)
        if out is None:
            dev = self.device
            out = dict(obs=torch.empty((K, n, 2, 3, 52), device=dev),
                       terminal_observation=torch.empty((K, n, 2, 3, 52), device=dev),
                       rew=torch.empty((K, n, 2, 3, 4), device=dev),
                       dones=torch.empty((K, n), device=dev, dtype=torch.long),
                       time_outs=torch.empty((K, n), device=dev, dtype=torch.bool),
                       progress_buffer=torch.empty((K, n), device=dev))
        rio = N.VssRolloutIO(actions.data_ptr(), out["obs"].data_ptr(), out["terminal_observation"].data_ptr(),
                             out["rew"].data_ptr(), out["dones"].data_ptr(), out["time_outs"].data_ptr(),
                             out["progress_buffer"].data_ptr())
        prm, st = self._c_params(), self._c_state()
        rc = N.load().vss_rollout(N.stream_of(self.device), n, K, N.ctypes.byref(prm), N.ctypes.byref(st),
                                  N.ctypes.byref(rio))
        N.check(rc, "vss_rollout")
        return out

    def _clipped(self, obs):
        if math.isinf(self.clip_obs):
            return obs
        return torch.clamp(obs, -self.clip_obs, self.clip_obs)

    def reset(self):
        """Ext VecTask.reset: the current observations (fields were reset at construction)."""
        self.obs_dict["obs"] = self._clipped(self.obs_buf)
        return self.obs_dict

    def reset_dones(self):
        """Re-sample every field whose `reset_buf` is set (envs/vss.py:267-333)."""
        prm, st = self._c_params(), self._c_state()
        rc = N.load().vss_reset_dones(N.stream_of(self.device), self.num_fields, N.ctypes.byref(prm),
                                      N.ctypes.byref(st))
        N.check(rc, "vss_reset_dones")

    def compute_observations(self, out: torch.Tensor | None = None, n_agents: int = 6):
        """compute_obs (envs/vss.py:205-216, 530-575) into `obs_buf` (or `out`)."""
        if n_agents not in (1, 3, 6):
            raise ValueError("n_agents must be 1 (blue robot 0), 3 (blue team) or 6 (both teams)")
        out = self.obs_buf if out is None else out
        self._check_buffer("out", out, self.num_fields * n_agents * 52, torch.float32)
        st = self._c_state()
        rc = N.load().vss_compute_observations(N.stream_of(self.device), self.num_fields, N.ctypes.byref(st),
                                               out.data_ptr(), n_agents)
        N.check(rc, "vss_compute_observations")
        return out

    def render(self, mode="rgb_array", env_id: int = 0, width: int = 400, height: int = 300):
        """Top-down RGB frame of field `env_id` (the Isaac Gym viewer capture behind capture_video,
        ppo…:213-221; envs/render.py); other modes (the interactive viewer) return None."""
        if mode != "rgb_array":
            return None
        from .render import render_field
        s = self.state[:, int(env_id)].detach().cpu().numpy().astype(np.float64)
        qz, qw = s[N.CH_RQZ:N.CH_RQZ + 6], s[N.CH_RQW:N.CH_RQW + 6]
        yaw = np.arctan2(2.0 * qw * qz, qw * qw - qz * qz)  # get_euler_xyz yaw with qx = qy = 0
        robots = np.stack([s[N.CH_RX:N.CH_RX + 6], s[N.CH_RY:N.CH_RY + 6], yaw], 1)
        return render_field(s[[N.CH_BALL_X, N.CH_BALL_Y]], robots, width, height)

    def close(self):
        pass
