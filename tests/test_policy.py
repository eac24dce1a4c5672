"""Fused rollout policy kernel (csrc/vss_policy.hip) vs the PyTorch Agent forward, fp32.

Tolerance: the kernel sums each dot product in a different order than hipBLASLt, otherwise
identical fp32 arithmetic (exact fp32 MFMA FMA chains) — relative 2e-5 on mean / value /
log-prob.  Sampled actions: mean + exp(logstd) * z with z ~ N(0, 1) (checked by moments)."""
from collections import namedtuple

import numpy as np
import pytest
import torch

import ppo_continuous_action_isaacgym as P
from envs._gym import Box

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
Env = namedtuple("Env", ["single_observation_space", "single_action_space"])


def make_agent(act_dim, seed):
    torch.manual_seed(seed)
    a = P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (act_dim,)))).to(DEV)
    with torch.no_grad():  # non-trivial last layers and log-std (init has 0.01-scaled actor outputs)
        a.actor_mean[8].weight.mul_(50.0)
        a.actor_logstd.fill_(-0.7)
        for m in a.modules():
            if isinstance(m, torch.nn.Linear):
                m.bias.uniform_(-0.1, 0.1)
    return a


# rows <= 4,096: policy_split_kernel (one 16-row group per workgroup, tiles split over its waves);
# 4,097-8,192: policy_kernel_both; larger: one launch per network (the rollout's chain path aside)
@pytest.mark.parametrize("act_dim,rows", [(2, 65536), (6, 4096), (2, 1), (2, 37), (6, 1000), (2, 4097), (6, 8192)])
def test_fused_forward_matches_agent(act_dim, rows):
    from vss_amd.policy import FusedPolicy
    agent = make_agent(act_dim, 7 + act_dim)
    fused = FusedPolicy(agent, seed=3)
    obs = torch.randn(rows, 52, device=DEV) * 0.7
    act = torch.randn(rows, act_dim, device=DEV) * 0.5
    with torch.no_grad():
        _, logp_t, ent_t, val_t = agent.get_action_and_value(obs, act)
        mean_t = agent.actor_mean(obs)
    a, logp, ent, val = fused.get_action_and_value(obs, act)
    torch.testing.assert_close(fused.actor_mean(obs), mean_t, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(val, val_t, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(logp, logp_t, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(ent, ent_t, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(fused.get_value(obs), val_t, rtol=2e-5, atol=2e-6)


def test_fused_sampling_statistics_and_logprob_consistency():
    from vss_amd.policy import FusedPolicy
    agent = make_agent(2, 1)
    fused = FusedPolicy(agent, seed=9)
    obs = torch.randn(65536, 52, device=DEV)
    a, logp, ent, val = fused.get_action_and_value(obs)
    mean = fused.actor_mean(obs)
    std = float(torch.exp(agent.actor_logstd[0, 0]))
    z = ((a - mean) / std).double()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    assert abs(((z ** 4).mean() / 3.0).item() - 1.0) < 0.03
    with torch.no_grad():
        _, logp_t, _, _ = agent.get_action_and_value(obs, a)
    torch.testing.assert_close(logp, logp_t, rtol=2e-5, atol=2e-5)
    a2, _, _, _ = fused.get_action_and_value(obs)
    assert not torch.equal(a, a2)  # fresh draws on every call


def test_refresh_tracks_parameter_updates():
    from vss_amd.policy import FusedPolicy
    agent = make_agent(2, 4)
    fused = FusedPolicy(agent)
    obs = torch.randn(256, 52, device=DEV)
    with torch.no_grad():
        for p in agent.parameters():
            p.add_(0.01 * torch.randn_like(p))
    fused.refresh()
    with torch.no_grad():
        want = agent.get_value(obs)
    torch.testing.assert_close(fused.get_value(obs), want, rtol=2e-5, atol=2e-6)


def test_refresh_tracks_parameter_updates_on_the_chain_path():
    """At rollout sizes (the GEMM chain) refresh() also renews the chain's x6 weight planes: after a
    parameter change and refresh() the values follow the new weights."""
    from vss_amd import policy as PM
    agent = make_agent(2, 6)
    fused = PM.FusedPolicy(agent)
    rows = PM.CHAIN_MIN_ROWS
    obs = torch.randn(rows, 52, device=DEV)
    assert fused.chain_active(rows)
    v0 = fused.get_value(obs)
    with torch.no_grad():
        for p in agent.parameters():
            p.add_(0.01 * torch.randn_like(p))
        want = agent.get_value(obs)
    assert not torch.allclose(v0, want, rtol=1e-4, atol=1e-5)
    fused.refresh()
    torch.testing.assert_close(fused.get_value(obs), want, rtol=2e-5, atol=2e-6)


def test_masked_terminal_values_write_only_masked_rows():
    from vss_amd.policy import FusedPolicy
    agent = make_agent(2, 5)
    fused = FusedPolicy(agent)
    rows = 4096 + 17
    obs = torch.randn(rows, 52, device=DEV)
    mask = torch.zeros(rows, dtype=torch.long, device=DEV)
    mask[torch.randperm(rows, device=DEV)[:100]] = 1
    mask[-3:] = 1
    out = torch.full((rows, 1), 7.0, device=DEV)
    fused.get_value_masked(obs, mask, out)
    full = fused.get_value(obs)
    m = mask.bool()
    assert torch.equal(out[m], full[m])             # bit-identical to the unmasked pass
    assert torch.all(out[~m] == 7.0)                # untouched elsewhere
    out0 = torch.full((rows, 1), 7.0, device=DEV)
    fused.get_value_masked(obs, torch.zeros_like(mask), out0)
    assert torch.all(out0 == 7.0)


def test_rejects_bad_shapes_before_launch():
    """The kernels trust their pointers: a network of the wrong shape, a short action or output
    buffer, or an output in the wrong dtype is refused on the host."""
    from vss_amd.policy import FusedPolicy
    agent = make_agent(2, 6)
    wrong = make_agent(2, 6)
    wrong.critic[2] = torch.nn.Linear(256, 500).to(DEV)
    with pytest.raises(ValueError):
        FusedPolicy(wrong)
    fused = FusedPolicy(agent)
    obs = torch.randn(64, 52, device=DEV)
    with pytest.raises(ValueError):
        fused.get_action_and_value(obs, torch.zeros(63, 2, device=DEV))
    mask = torch.ones(64, dtype=torch.long, device=DEV)
    with pytest.raises(ValueError):
        fused.get_value_masked(obs, mask, torch.zeros(63, 1, device=DEV))
    with pytest.raises(ValueError):
        fused.get_value_masked(obs, mask, torch.zeros(64, 1, device=DEV, dtype=torch.float64))
    out = torch.zeros(64, 1, device=DEV)
    fused.get_value_masked(obs, mask.bool(), out)  # a bool mask (the env's dones) is accepted
    assert torch.equal(out, fused.get_value(obs))


def test_outputs_written_into_caller_buffers():
    """The rollout form (ppo…:262-266 into the storage rows): out=(action, logprob, value) buffers are
    written in place, with the same values as the allocating form; the entropy is not computed."""
    from vss_amd.policy import FusedPolicy
    agent = make_agent(2, 8)
    fused = FusedPolicy(agent, seed=4)
    obs = torch.randn(4096 + 7, 52, device=DEV)
    act = torch.randn(obs.shape[0], 2, device=DEV) * 0.5
    store_a = torch.zeros((3, obs.shape[0], 2), device=DEV)
    store_lp = torch.zeros((3, obs.shape[0]), device=DEV)
    store_v = torch.zeros((3, obs.shape[0]), device=DEV)
    a, lp, ent, v = fused.get_action_and_value(obs, act, out=(store_a[1], store_lp[1], store_v[1].view(-1, 1)))
    assert ent is None and lp.data_ptr() == store_lp[1].data_ptr() and v.data_ptr() == store_v[1].data_ptr()
    _, lp2, _, v2 = fused.get_action_and_value(obs, act)
    assert torch.equal(store_lp[1], lp2) and torch.equal(store_v[1], v2.view(-1))
    assert torch.all(store_lp[0] == 0) and torch.all(store_lp[2] == 0)
    a3, _, _, _ = fused.get_action_and_value(obs, out=(store_a[2], store_lp[2], store_v[2].view(-1, 1)))
    assert a3.data_ptr() == store_a[2].data_ptr() and not torch.all(store_a[2] == 0)
    with torch.no_grad():
        _, lp_t, _, _ = agent.get_action_and_value(obs, store_a[2])
    torch.testing.assert_close(store_lp[2], lp_t, rtol=2e-5, atol=2e-5)
    with pytest.raises(ValueError):
        fused.get_action_and_value(obs, out=(store_a[2], store_lp[2][:-1], store_v[2].view(-1, 1)))


def test_chain_path_matches_fused_kernel_and_agent():
    """At rollout sizes the policy runs as the GEMM chain (first layer fp32 MFMA, hidden layers x6,
    output folded) + vss_policy_sample: means / values within fp32 rounding of the fused kernel and of
    the torch Agent, the same Philox draws (action - mean identical in distribution: with the same
    seed and counter, the z of both paths agree to the means' rounding), entropy identical."""
    from vss_amd import policy as PM
    agent = make_agent(2, 21)
    rows = PM.CHAIN_MIN_ROWS * 2
    obs = torch.randn(rows, 52, device=DEV) * 0.7
    chain, fused = PM.FusedPolicy(agent, seed=5), PM.FusedPolicy(agent, seed=5)
    assert chain.chain_active(rows)
    a_c, lp_c, ent_c, v_c = chain.get_action_and_value(obs)
    mean_c = chain.actor_mean(obs)
    old = PM.ROLLOUT_POLICY
    try:
        PM.ROLLOUT_POLICY = "fused"
        a_f, lp_f, ent_f, v_f = fused.get_action_and_value(obs)
        mean_f = fused.actor_mean(obs)
    finally:
        PM.ROLLOUT_POLICY = old
    with torch.no_grad():
        mean_t, v_t = agent.actor_mean(obs), agent.get_value(obs)
    torch.testing.assert_close(mean_c, mean_t, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(mean_c, mean_f, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(v_c, v_t, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(v_c, v_f, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(a_c - mean_c, a_f - mean_f, rtol=0, atol=1e-5)  # same z
    torch.testing.assert_close(lp_c, lp_f, rtol=2e-5, atol=2e-5)
    assert torch.equal(ent_c, ent_f)
    vr = chain.values_chain(obs[:1000])  # any row count: the same per-row values
    assert torch.equal(vr, v_c[:1000])
