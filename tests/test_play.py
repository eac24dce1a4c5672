"""play.py drop-in (play_matches + teams, play.py:26-164) on the HIP env."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def make_env(n, max_len):
    from envs.vss import VSS, default_cfg
    cfg = default_cfg(n)
    cfg["env"]["maxEpisodeLength"] = max_len
    cfg["env"]["seed"] = 321
    env = VSS(cfg, DEV, DEV, 0, True, False, False)
    env.w_goal, env.w_grad, env.w_move, env.w_energy = 1.0, 0.0, 0.0, 0.0  # ppo…:389-392
    return env


def oracle_play_zero(env_seed, n, max_len, n_matches):
    """The reference's play_matches loop (play.py:131-164), zero teams, on the CPU oracle."""
    h = O.HostEnv(n)
    prm = O.params(1.0, 0.0, 0.0, 0.0, 1.0, max_len, env_seed)
    O.reset_dones(h, prm)          # construction
    h.reset[:] = 1
    O.reset_dones(h, prm)          # envs.reset_buf[:] = 1; envs.reset_dones()
    io = O.make_io(n, O.MODE_FULL)
    zero = np.zeros((n, 12), np.float32)
    ep, rs, ls = 0, 0.0, 0.0
    while ep < n_matches:
        O.step(h, O.MODE_FULL, zero, io, prm)
        ids = np.nonzero(h.reset[:1065])[0]
        if len(ids):
            ep += len(ids)
            rs += float(io["rew"].reshape(n, 2, 3, 4)[ids, 0, 0, 0].sum())
            ls += float(io["progress_f"][ids].sum())
    return rs / ep, ls / ep


def test_play_zero_vs_zero_matches_oracle():
    from play import get_team, play_matches
    n, max_len = 1100, 30
    env = make_env(n, max_len)
    got = play_matches(env, get_team("zero"), get_team("zero"), 1500)
    want = oracle_play_zero(321, n, max_len, 1500)
    assert got == pytest.approx(want, abs=0, rel=0)


def test_play_with_agent_checkpoints(tmp_path):
    """ppo-sa / ppo-sa-x3 / ppo-cma / ppo-dma teams load state-dict checkpoints (weights_only)."""
    from collections import namedtuple
    from envs._gym import Box
    from play import get_team, play_matches
    import ppo_continuous_action_isaacgym as P
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    paths = {}
    for adim in (2, 6):
        torch.manual_seed(adim)
        a = P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (adim,))))
        paths[adim] = str(tmp_path / f"agent{adim}.pt")
        torch.save(a.state_dict(), paths[adim])
    env = make_env(2048, 40)
    for algo, adim in (("ppo-sa", 2), ("ppo-sa-x3", 2), ("ppo-cma", 6), ("ppo-dma", 2)):
        score, length = play_matches(env, get_team(algo, paths[adim]), get_team("ou"), 500)
        assert -1.0 <= score <= 1.0 and 1.0 <= length <= 40.0, (algo, score, length)
