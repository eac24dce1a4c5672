#!/usr/bin/env python3
"""Profiling-only: the rollout's actor + critic forward at ROWS = 65,536 as a chain of the update's
GEMM kernels (first layer fp32 MFMA, hidden layers bf16x6, output layer folded into the last launch)
against the fused rollout policy kernel (csrc/vss_policy.hip)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from vss_amd.policy import FusedPolicy  # noqa: E402
from vss_amd.update import linear_tanh, linear_tanh_mixed as linear_tanh_x6, linear_tanh_out_mixed as linear_tanh_out_x6  # noqa: E402

from collections import namedtuple  # noqa: E402

import numpy as np  # noqa: E402
from envs._gym import Box  # noqa: E402

rows = int(os.environ.get("ROWS", 65536))
torch.manual_seed(0)
Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
agent = P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (2,)))).cuda()
obs = torch.randn(rows, 52, device="cuda")
fused = FusedPolicy(agent)


def chain(seq):
    lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
    h = linear_tanh(obs, lin[0].weight, lin[0].bias)
    h = linear_tanh_x6(h, lin[1].weight, lin[1].bias)
    h = linear_tanh_x6(h, lin[2].weight, lin[2].bias)
    return linear_tanh_out_x6(h, lin[3].weight, lin[3].bias, lin[4].weight, lin[4].bias)[1]


def timeit(fn, reps=50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    t_chain = timeit(lambda: (chain(agent.actor_mean), chain(agent.critic)))
    from vss_amd import policy as PM
    old, PM.ROLLOUT_POLICY = PM.ROLLOUT_POLICY, "fused"
    t_fused = timeit(lambda: fused.get_action_and_value(obs))
    PM.ROLLOUT_POLICY = old
    t_path = timeit(lambda: fused.get_action_and_value(obs))
    m_ref = agent.actor_mean(obs)
    print(f"rows {rows}: x6 chain actor+critic {t_chain:.3f} ms, fused policy kernel {t_fused:.3f} ms; "
          f"rollout path (chain + vss_policy_sample) {t_path:.3f} ms; chain mean max|diff| vs torch {float((chain(agent.actor_mean) - m_ref).abs().max()):.2e}", flush=True)
