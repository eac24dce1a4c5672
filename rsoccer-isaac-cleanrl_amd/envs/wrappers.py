"""Drop-in wrappers of the reference's envs/wrappers.py, fused into the HIP step.

`SingleAgent`, `CMA` and `DMA` keep the reference's behaviour (envs/wrappers.py:89-180): the
robots the learner does not control are driven by Ornstein-Uhlenbeck noise on the wrapper's
`action_buf` (random_ou, envs/wrappers.py:5-19), the learner's actions overwrite their slots,
the step runs, `action_buf` is zeroed for finished fields, and observations / rewards are sliced
to the learner's view.  Here all of that happens inside the single `vss_step` launch
(VSS_MODE_SA/CMA/DMA): the OU noise is drawn by the kernel's Philox stream, and only the
learner's rows are written to HBM — no (N,2,3,52) observation tensor, no host sync on `dones`.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from vss_amd import _native as N

from ._gym import Box, Wrapper
from .vss import VSS, default_cfg


def random_ou(prev: torch.Tensor) -> torch.Tensor:
    """One OU step on an action buffer: clamp(prev - 0.1 prev + N(0, 0.15^2), -1, 1).

    Same update as the reference's random_ou (envs/wrappers.py:5-19) in plain torch, for
    callers that drive their own action buffers (e.g. play.py's TeamOU); the wrappers below do
    it inside the HIP step."""
    theta, sigma = 0.1, 0.15
    noise = torch.randn(prev.shape, device=prev.device, dtype=prev.dtype) * sigma
    return (prev - theta * prev + noise).clamp(-1.0, 1.0)


def _local_device() -> str:
    # one process per GPU: LOCAL_RANK; VSS_LOCAL_DEVICE pins it (several ranks on one GPU)
    return f"cuda:{int(os.environ.get('VSS_LOCAL_DEVICE', os.environ.get('LOCAL_RANK', 0)))}"


def make_env(args):
    """(unwrapped VSS, wrapped env) for args.env_id in {sa, cma, dma} (envs/wrappers.py:21-48)."""
    assert args.cuda
    cfg = default_cfg(args.num_envs)
    if args.env_id == "dma":
        assert args.num_envs % 3 == 0
        cfg["env"]["numEnvs"] = int(args.num_envs / 3)
    if getattr(args, "seed", None) is not None:
        cfg["env"]["seed"] = int(args.seed) * 1000003 + int(os.environ.get("RANK", 0))
    device = _local_device()
    envs = VSS(cfg=cfg, rl_device=device, sim_device=device, graphics_device_id=0,
               headless=not getattr(args, "capture_video", False),
               virtual_screen_capture=getattr(args, "capture_video", False), force_render=False)
    wrappers = {"sa": SingleAgent, "cma": CMA, "dma": DMA}
    return envs, wrappers[args.env_id](envs)


class RecordEpisodeStatisticsTorch(Wrapper):
    """Running per-env returns (goal, grad, move, energy) and lengths (envs/wrappers.py:50-87),
    updated by one HIP launch per step (`vss_episode_stats`) instead of seven elementwise ops."""

    def __init__(self, env, device):
        super().__init__(env)
        self.num_envs = getattr(env, "num_envs", 1)
        self.device = N.require_device(device)
        self.episode_returns = None
        self.episode_lengths = None

    def reset(self, **kwargs):
        observations = super().reset(**kwargs)
        n = self.num_envs
        self.episode_returns = torch.zeros((n, 4), dtype=torch.float32, device=self.device)
        self.episode_lengths = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.returned_episode_returns = torch.zeros_like(self.episode_returns)
        self.returned_episode_lengths = torch.zeros_like(self.episode_lengths)
        self.returned_return_sum = torch.zeros(n, dtype=torch.float32, device=self.device)
        return observations

    def step(self, action):
        observations, rewards, dones, infos = super().step(action)
        rews = infos["rews"]
        n = self.num_envs
        if (rews.shape != (n, 4) or rews.dtype != torch.float32 or not rews.is_contiguous()
                or dones.numel() != n or dones.dtype != torch.long or not dones.is_contiguous()):
            raise ValueError("episode statistics expect rews (N, 4) float32 and dones (N,) int64, contiguous")
        N.check(N.load().vss_episode_stats(
            N.stream_of(self.device), n, rews.data_ptr(), dones.data_ptr(), self.episode_returns.data_ptr(),
            self.episode_lengths.data_ptr(), self.returned_episode_returns.data_ptr(),
            self.returned_episode_lengths.data_ptr(), self.returned_return_sum.data_ptr()), "vss_episode_stats")
        r = self.returned_episode_returns
        infos["r"] = {"goal": r[:, 0], "grad": r[:, 1], "move": r[:, 2], "energy": r[:, 3],
                      "return": self.returned_return_sum}
        infos["l"] = self.returned_episode_lengths
        return observations, rewards, dones, infos


class _FusedWrapper(Wrapper):
    """Common part of SA / CMA / DMA: the OU action buffer and the packed output buffers."""

    MODE = None
    LEARNER_WIDTH = 2  # floats per learner row
    ROWS_PER_FIELD = 1  # learner rows per field

    def __init__(self, env: VSS):
        super().__init__(env)
        self.action_buf = env.dof_velocity_buf.clone()  # (N,2,3,2) OU state
        n, dev = env.num_fields, env.device
        rows = n * self.ROWS_PER_FIELD
        self._obs = torch.zeros((rows, env.num_obs), device=dev)
        self._terminal_obs = torch.zeros_like(self._obs)
        self._rews = torch.zeros((rows, 4), device=dev)
        self._reward = torch.zeros(rows, device=dev)
        if self.ROWS_PER_FIELD == 1:
            self._time_outs, self._progress = env.timeout_buf, env.progress_f_buf
            self._dones = None
        else:
            self._time_outs = torch.zeros(rows, dtype=torch.bool, device=dev)
            self._progress = torch.zeros(rows, device=dev)
            self._dones = torch.zeros(rows, dtype=torch.long, device=dev)
        env.compute_observations(self._obs, n_agents=3 if self.ROWS_PER_FIELD == 3 else 1)

    def _first_obs(self):
        self.env.compute_observations(self._obs, n_agents=3 if self.ROWS_PER_FIELD == 3 else 1)
        return {"obs": self._obs}

    def reset(self, **kwargs):
        self.env.reset(**kwargs)
        return self._first_obs()

    def _rews_view(self):
        return self._rews

    def step(self, action):
        env = self.env
        env.native_step(self.MODE, action, dict(
            ou_buf=self.action_buf, obs=self._obs, terminal_obs=self._terminal_obs, rew=self._rews,
            reward_sum=self._reward, dones_rep=self._dones, time_outs=self._time_outs,
            progress_f=self._progress))
        infos = {"rews": self._rews_view(), "terminal_observation": self._terminal_obs,
                 "time_outs": self._time_outs, "progress_buffer": self._progress}
        dones = env.reset_buf if self._dones is None else self._dones
        return {"obs": self._obs}, self._reward, dones, infos


class SingleAgent(_FusedWrapper):
    """Learner = blue robot 0; the other five robots follow OU noise (envs/wrappers.py:89-115)."""

    MODE = N.MODE_SA

    def __init__(self, env):
        super().__init__(env)
        self._action_space = Box(-1.0, 1.0, (env.num_actions,))
        self._observation_space = Box(-np.inf, np.inf, (env.num_obs,))
        self.act_view = self.action_buf[:, 0, 0, :]


class CMA(_FusedWrapper):
    """Centralised multi-agent: one 6-vector drives the blue team (envs/wrappers.py:118-148)."""

    MODE = N.MODE_CMA

    def __init__(self, env):
        super().__init__(env)
        self.num_envs = getattr(env, "num_envs", 1)
        self.device = env.device
        num_actions = env.num_actions * 3
        self._action_space = Box(-1.0, 1.0, (num_actions,))
        self._observation_space = Box(-np.inf, np.inf, (env.num_obs,))
        self.act_view = self.action_buf[:, 0, :, :].view(-1, num_actions)


class DMA(_FusedWrapper):
    """Decentralised multi-agent: each blue robot is one learner row (envs/wrappers.py:151-180)."""

    MODE = N.MODE_DMA
    ROWS_PER_FIELD = 3

    def __init__(self, env):
        setattr(env, "num_environments", getattr(env, "num_envs", 1) * 3)
        super().__init__(env)
        self._action_space = Box(-1.0, 1.0, (env.num_actions,))
        self._observation_space = Box(-np.inf, np.inf, (env.num_obs,))
