"""Fused rollout policy: the reference Agent's forward (ppo_continuous_action_isaacgym.py:154-164)
as one HIP kernel on the fp32 matrix cores (csrc/vss_policy.hip, include/vss.h `vss_policy_forward`).

    fused = FusedPolicy(agent)          # packs actor + critic weights (lane order) on the device
    fused.refresh()                     # after every optimizer step (weights changed)
    action, logprob, entropy, value = fused.get_action_and_value(obs)
    value = fused.get_value(obs)

Results equal the torch Agent's within fp32 summation-order rounding (tests/test_policy.py);
actions are sampled from the same Normal(mean, exp(logstd)) with a Philox stream instead of
torch's generator.  Inference only (no autograd): the PPO update keeps the torch modules.

At rollout sizes (>= CHAIN_MIN_ROWS rows, e.g. 65,536 envs) the two forwards run instead as a chain
of the update's GEMM kernels -- first layer on the fp32 MFMA kernel, the 256/512-wide layers in fp32
arithmetic on the bf16 matrix cores (csrc/vss_gemm_x6.hip, output layer folded into the last launch)
-- and vss_policy_sample draws the actions from the actor means with the fused kernel's Philox
stream: 0.93 ms instead of 1.21 ms for actor + critic at 65,536 rows (profiles/r03o_*).  Smaller
batches keep the single fused launch.  VSS_ROLLOUT_POLICY=fused forces the fused kernel.  The chain's
bf16 weight planes are made once per refresh(), like the fused kernel's packed weights: both evaluate
the weights as of the last refresh().
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native as N
from .update import linear_tanh_mixed, linear_tanh_out_mixed, weight_planes, x6_ok

CHAIN_MIN_ROWS = 16384
ROLLOUT_POLICY = os.environ.get("VSS_ROLLOUT_POLICY", "chain")


class FusedPolicy:
    def __init__(self, agent, seed: int = 0):
        self.agent = agent
        self.device = next(agent.parameters()).device
        N.require_device(self.device)
        self.n_act = int(agent.actor_logstd.shape[-1])
        if self.n_act not in (2, 6):
            raise ValueError("fused policy supports 2 (SA/DMA) or 6 (CMA) actions")
        lib = N.load()
        self._actor = torch.empty(lib.vss_mlp_packed_size(self.n_act), device=self.device)
        self._critic = torch.empty(lib.vss_mlp_packed_size(1), device=self.device)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0
        self._keep = {}
        self.refresh()

    @staticmethod
    def _linears(seq):
        return [m for m in seq if isinstance(m, torch.nn.Linear)]

    def _pack(self, seq, n_out, out):
        lins = self._linears(seq)
        dims = [52, 256, 512, 512, 256, n_out]
        if len(lins) != 5 or any((l.in_features, l.out_features) != (dims[i], dims[i + 1]) for i, l in enumerate(lins)):
            raise ValueError(f"expected the reference Agent's MLP {' -> '.join(map(str, dims))}")
        ws = [l.weight.detach().to(self.device, torch.float32).contiguous() for l in lins]
        bs = [l.bias.detach().to(self.device, torch.float32).contiguous() for l in lins]
        self._keep[n_out] = ws + bs  # alive until the (asynchronous) pack has read them
        wa = (ctypes.c_void_p * 5)(*[w.data_ptr() for w in ws])
        ba = (ctypes.c_void_p * 5)(*[b.data_ptr() for b in bs])
        N.check(N.load().vss_mlp_pack(N.stream_of(self.device), n_out, wa, ba, out.data_ptr()), "vss_mlp_pack")

    @torch.no_grad()
    def refresh(self):
        """Re-pack the current actor / critic weights (call after optimizer.step()): the fused kernel's
        packed weights and the GEMM chain's bf16 weight planes (one vss_weight_planes_bf16x6 launch for
        both MLPs' hidden layers, instead of a split launch per layer and rollout step)."""
        self._pack(self.agent.actor_mean, self.n_act, self._actor)
        self._pack(self.agent.critic, 1, self._critic)
        self._planes = {}
        if ROLLOUT_POLICY == "chain":
            jobs = [(id(seq), i, m.weight.detach()) for seq in (self.agent.actor_mean, self.agent.critic)
                    for i, m in enumerate(self._linears(seq)[1:-1], 1)
                    if m.weight.dtype == torch.float32 and m.weight.is_contiguous()
                    and x6_ok(256, m.in_features, m.out_features)]
            if jobs:
                planes = weight_planes([(w, False) for _, _, w in jobs])
                self._planes = {(k, i): p for (k, i, _), p in zip(jobs, planes)}

    def _chain(self, seq, obs):
        """One MLP's output (rows, n_out) through the update's GEMM kernels (no autograd)."""
        lins = self._linears(seq)
        h = obs
        pl = self._planes
        for i, m in enumerate(lins[:-2]):
            h = linear_tanh_mixed(h, m.weight.detach(), m.bias.detach(), planes=pl.get((id(seq), i)))
        return linear_tanh_out_mixed(h, lins[-2].weight.detach(), lins[-2].bias.detach(), lins[-1].weight.detach(),
                                     lins[-1].bias.detach(), planes=pl.get((id(seq), len(lins) - 2)))[1]

    def chain_active(self, rows: int) -> bool:
        """Whether a batch of `rows` observations is evaluated by the GEMM chain."""
        return ROLLOUT_POLICY == "chain" and rows >= CHAIN_MIN_ROWS

    @torch.no_grad()
    def values_chain(self, obs):
        """critic(obs) through the GEMM chain for ANY row count, padded to whole 256-row tiles so every
        row takes the same kernels as in a chain-sized batch: a row's value does not depend on the
        batch it is evaluated in (the masked terminal pass of the rollout relies on it)."""
        obs = obs.reshape(-1, 52).to(self.device, torch.float32)
        rows = obs.shape[0]
        pad = -rows % 256
        if pad:
            obs = torch.cat([obs, obs.new_zeros((pad, 52))])
        return self._chain(self.agent.critic, obs.contiguous())[:rows]

    def _run(self, obs, actor: bool, action=None, out=None, want_mean=False):
        obs = obs.reshape(-1, 52)
        if obs.dtype != torch.float32 or not obs.is_contiguous() or obs.device != self.device:
            obs = obs.to(self.device, torch.float32).contiguous()
        rows = obs.shape[0]
        dev = self.device
        if ROLLOUT_POLICY == "chain" and rows >= CHAIN_MIN_ROWS:
            return self._run_chain(obs, actor, action, out, want_mean)
        if out is not None:
            # caller-owned outputs (the rollout storage rows): action, log-prob and value written in place
            act_out, logp, value = out
            for t, w in ((act_out, rows * self.n_act), (logp, rows), (value, rows)):
                if t.numel() != w or t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
                    raise ValueError("out buffers must be contiguous fp32 on the policy's device with one row per obs")
            outs = [act_out if action is None else None, logp, None, None]
        else:
            value = torch.empty((rows, 1), device=dev)
            outs = [None] * 4
            if actor:
                outs = [torch.empty((rows, self.n_act), device=dev) if action is None else None,
                        torch.empty(rows, device=dev), torch.empty(rows, device=dev),
                        torch.empty((rows, self.n_act), device=dev) if want_mean else None]
        if actor and action is not None:
            action = action.to(dev, torch.float32).contiguous()
            if action.numel() != rows * self.n_act:
                raise ValueError(f"action must have {rows} x {self.n_act} elements, got {tuple(action.shape)}")
        self.counter += 1
        rc = N.load().vss_policy_forward(
            N.stream_of(dev), rows, self.n_act, obs.data_ptr(), self._actor.data_ptr() if actor else None,
            self.agent.actor_logstd.detach().data_ptr(), self._critic.data_ptr(), self.seed, self.counter,
            N.ptr(action), N.ptr(outs[0]), N.ptr(outs[1]), N.ptr(outs[2]), value.data_ptr(), N.ptr(outs[3]))
        N.check(rc, "vss_policy_forward")
        if actor:
            return (action if action is not None else outs[0]), outs[1], outs[2], value, outs[3]
        return value

    def _run_chain(self, obs, actor: bool, action, out, want_mean):
        """_run through the GEMM chain + vss_policy_sample (same outputs and sampling stream)."""
        rows, dev = obs.shape[0], self.device
        value = self._chain(self.agent.critic, obs)
        if not actor:
            return value
        mean = self._chain(self.agent.actor_mean, obs).contiguous()
        if out is not None:
            act_out, logp, val_out = out
            for t, w in ((act_out, rows * self.n_act), (logp, rows), (val_out, rows)):
                if t.numel() != w or t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
                    raise ValueError("out buffers must be contiguous fp32 on the policy's device with one row per obs")
            val_out.view(rows, 1).copy_(value)
            value, ent = val_out, None
            act_out = act_out if action is None else None
        else:
            act_out = torch.empty((rows, self.n_act), device=dev) if action is None else None
            logp, ent = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        if action is not None:
            action = action.to(dev, torch.float32).contiguous()
            if action.numel() != rows * self.n_act:
                raise ValueError(f"action must have {rows} x {self.n_act} elements, got {tuple(action.shape)}")
        self.counter += 1
        N.check(N.load().vss_policy_sample(N.stream_of(dev), rows, self.n_act, mean.data_ptr(),
                                           self.agent.actor_logstd.detach().data_ptr(), self.seed, self.counter,
                                           N.ptr(action), N.ptr(act_out), logp.data_ptr(), N.ptr(ent)),
                "vss_policy_sample")
        return (action if action is not None else act_out), logp, ent, value, (mean if want_mean else None)

    @torch.no_grad()
    def get_action_and_value(self, obs, action=None, out=None):
        """Agent.get_action_and_value.  out = (action, logprob, value) buffers to write in place (the
        rollout storage rows; the entropy, which the rollout does not use, is then not computed and
        returned as None)."""
        a, logp, ent, value, _ = self._run(obs, True, action, out)
        return a, logp, ent, value

    @torch.no_grad()
    def get_value(self, obs):
        return self._run(obs, False)

    @torch.no_grad()
    def get_value_masked(self, obs, mask: torch.Tensor, out: torch.Tensor):
        """critic(obs) written into `out` (rows, 1) only for rows with mask != 0 (int64 mask,
        e.g. the env's dones); other rows of `out` are left untouched."""
        obs = obs.reshape(-1, 52).to(self.device, torch.float32).contiguous()
        rows = obs.shape[0]
        mask = mask.to(self.device, torch.long).contiguous()
        if (out.numel() != rows or out.dtype != torch.float32 or out.device != self.device
                or not out.is_contiguous() or mask.numel() != rows):
            raise ValueError("out (float32, contiguous, on the policy's device) and mask need one element per row")
        rc = N.load().vss_value_forward_masked(
            N.stream_of(self.device), rows, self.n_act, obs.data_ptr(), None, None,
            self._critic.data_ptr(), self.seed, 0, None, None, None, None, out.data_ptr(), None, mask.data_ptr())
        N.check(rc, "vss_value_forward_masked")
        return out

    @torch.no_grad()
    def actor_mean(self, obs):
        return self._run(obs, True, want_mean=True)[4]


class TerminalValues:
    """next_values[t] = critic(terminal_obs_t) (ppo…:272) for the fused rollout, in ONE masked critic
    pass after the rollout instead of a critic pass per step.  For a field that did not reset at
    step t the terminal observation IS next_obs_t, whose value the next step computes (values[t+1],
    or critic(next_obs) after the last step), so only the reset rows need the terminal pass; the
    critic does not change within a rollout, so one pass over all T x E recorded terminal
    observations, masked by the dones, gives the same values.  (A masked pass per step cost
    ~0.22 ms however few rows reset -- one wave's serial walk through the critic.)  Memory: the
    (T, E, obs) fp32 copy of the terminal observations, 1.7 GB at T = 128, E = 65,536 and 5.1 GB
    for DMA at 196,608 agent rows (<= 2 % of one MI355X's 288 GB)."""

    def __init__(self, T, E, obs_shape, device):
        self.T, self.E = T, E
        self.term_obs = torch.zeros((T, E) + tuple(obs_shape), device=device)
        self.term_mask = torch.zeros((T, E), device=device, dtype=torch.long)
        self.term_values = torch.zeros((T, E), device=device)

    def record(self, step, terminal_obs, done):
        self.term_obs[step].copy_(terminal_obs.reshape(self.term_obs.shape[1:]))
        self.term_mask[step].copy_(done)

    def next_values(self, fused, values, next_dones, next_obs):
        """(T, E) next_values: the masked terminal pass where a field reset, else values[t + 1].  When
        the rollout's values come from the GEMM chain (FusedPolicy.chain_active), the reset rows are
        gathered and evaluated by the same chain (one host sync for their count, once per rollout), so
        next_values stays exactly critic(terminal_obs) of one evaluator."""
        if fused.chain_active(self.E):
            idx = self.term_mask.view(-1).nonzero().squeeze(1)
            tv = self.term_values.view(-1)
            if idx.numel():
                tv.index_copy_(0, idx, fused.values_chain(self.term_obs.view(self.T * self.E, -1).index_select(0, idx))
                               .view(-1))
        else:
            fused.get_value_masked(self.term_obs, self.term_mask, self.term_values.view(self.T * self.E, 1))
        v_last = fused.get_value(next_obs).view(1, self.E)
        return torch.where(next_dones.bool(), self.term_values, torch.cat([values[1:], v_last], 0))
