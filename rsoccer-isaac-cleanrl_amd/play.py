"""Evaluation drop-in (the reference's play.py): team policies and `play_matches`.

`play_matches(envs, blue_team, yellow_team, n_matches)` plays the raw VSS env (no wrapper) with
one policy per team until `n_matches` episodes have finished among the first 1,065 fields, and
returns (mean blue goal score, mean episode length) — play.py:131-164.  Same result as the
reference's loop, but without its per-step host synchronisation: steps run in chunks, per-step
tallies stay on the device, and the host finds the exact step at which the reference would have
stopped, counting nothing after it.

Teams (play.py:26-102): 'zero', 'ou', and checkpoints of 'ppo-sa' / 'ppo-sa-x3' / 'ppo-cma' /
'ppo-dma' agents.  Checkpoints are loaded with `torch.load(weights_only=True)`.  The reference's
BASELINE_TEAMS point at base_nets/*.pt files that are not part of the reference snapshot
(.MISSING_LARGE_BLOBS); `baseline_teams()` returns whichever of them exist plus zero/ou.
"""
from __future__ import annotations

import os
from abc import ABC, abstractmethod
from collections import namedtuple

import numpy as np
import torch

from envs._gym import Box
from envs.wrappers import random_ou
from ppo_continuous_action_isaacgym import Agent

COUNT_FIELDS = 1065  # play.py:158 counts dones among the first 1065 fields (test.py:35)


class Team(ABC):
    def __init__(self, path=None, env_d=None):
        pass

    @abstractmethod
    def __call__(self, act, obs):
        """Write this team's (N,3,2) actions into `act` in place, from its (N,3,52) obs."""


class TeamZero(Team):
    def __call__(self, act, obs):
        act.mul_(0)


class TeamOU(Team):
    def __call__(self, act, obs):
        act.copy_(random_ou(act))


class TeamAgent(Team):
    def __init__(self, path, env_d, device="cuda:0"):
        self.agent = Agent(env_d).to(device)
        self.agent.load_state_dict(torch.load(path, map_location=device, weights_only=True))
        self.agent.eval()

    @torch.no_grad()
    def act(self, obs):
        return self.agent.get_action_and_value(obs)[0]


class TeamSA(TeamAgent):
    """One SA policy drives robot 0; robots 1-2 follow OU noise (play.py:51-54)."""

    def __call__(self, act, obs):
        act.copy_(random_ou(act))
        act[:, 0, :] = self.act(obs[:, 0, :])


class TeamCMA(TeamAgent):
    def __call__(self, act, obs):
        act.copy_(self.act(obs[:, 0, :]).view(-1, 3, 2))


class TeamDMA(TeamAgent):
    """Each robot acts on its own observation (play.py:62-64; also 'ppo-sa-x3')."""

    def __call__(self, act, obs):
        n = obs.shape[0]
        act.copy_(self.act(obs.reshape(n * 3, -1)).view(n, 3, 2))


def get_team(algo, path=None, device="cuda:0"):
    Dummy = namedtuple("dummy_env", ["single_observation_space", "single_action_space"])
    obs_space = Box(-np.inf, np.inf, (52,))
    if algo in ("ppo-sa", "ppo-sa-x3", "ppo-dma"):
        env_d = Dummy(obs_space, Box(-1.0, 1.0, (2,)))
        return (TeamSA if algo == "ppo-sa" else TeamDMA)(path, env_d, device)
    if algo == "ppo-cma":
        return TeamCMA(path, Dummy(obs_space, Box(-1.0, 1.0, (6,))), device)
    if algo == "zero":
        return TeamZero()
    if algo == "ou":
        return TeamOU()
    raise ValueError(f"Unknown algo: {algo}")


def baseline_teams(root="base_nets", device="cuda:0"):
    """The reference's BASELINE_TEAMS (play.py:105-128), restricted to checkpoints present."""
    teams = {}
    for algo, tag in (("ppo-sa", "ppo-sa"), ("ppo-sa-x3", "ppo-sa"), ("ppo-cma", "ppo-cma"), ("ppo-dma", "ppo-dma")):
        for seed in ("10", "20", "30"):
            p = os.path.join(root, f"exp000_{tag}_{seed}", "agent.pt")
            if os.path.exists(p):
                teams.setdefault(algo, {})[seed] = get_team(algo, p, device)
    teams["zero"] = {"00": get_team("zero")}
    teams["ou"] = {"00": get_team("ou")}
    return teams


@torch.no_grad()
def play_matches(envs, blue_team, yellow_team, n_matches, video_path=None, chunk=32):
    """Mean blue goal score and episode length over the first `n_matches` finished episodes."""
    envs.reset_buf[:] = 1
    envs.reset_dones()  # like the reference, obs_buf is not recomputed here (play.py:132-151)
    n = envs.num_fields
    k = min(COUNT_FIELDS, n)
    action_buf = torch.zeros((n,) + tuple(envs.action_space.shape), device=envs.device)
    obs = envs.reset()["obs"]
    rec = None
    if video_path:  # play.py:134-142: the first 300 steps of field 0 (envs/render.py, GIF)
        from envs.render import FrameRecorder
        rec = FrameRecorder(lambda: envs.render("rgb_array"), video_path, lambda step: step == 0, 300, "video.000")
    ep_count, rew_sum, len_sum = 0, 0.0, 0.0
    while ep_count < n_matches:
        cnt = torch.zeros(chunk, device=envs.device, dtype=torch.int64)
        rsum = torch.zeros(chunk, device=envs.device, dtype=torch.float64)
        lsum = torch.zeros(chunk, device=envs.device, dtype=torch.float64)
        for t in range(chunk):
            blue_team(action_buf[:, 0], obs[:, 0])
            yellow_team(action_buf[:, 1], obs[:, 1])
            o, rew, dones, info = envs.step(action_buf)
            if rec is not None:
                rec.on_step()
            obs = o["obs"]
            d = dones[:k] != 0
            cnt[t] = d.sum()
            rsum[t] = (rew[:k, 0, 0, 0] * d).sum()
            lsum[t] = (info["progress_buffer"][:k] * d).sum()
        c, r, l = cnt.cpu().numpy(), rsum.cpu().numpy(), lsum.cpu().numpy()
        for t in range(chunk):  # replay the reference's per-step stopping rule on the host
            if ep_count >= n_matches:
                break
            if c[t]:
                ep_count += int(c[t])
                rew_sum += float(r[t])
                len_sum += float(l[t])
    if rec is not None:
        rec.flush()
    return rew_sum / ep_count, len_sum / ep_count
