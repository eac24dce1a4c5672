"""Drop-in PPO train loop (cleanrl ppo_continuous_action_isaacgym, as used by the reference's
ppo_continuous_action_isaacgym.py) on the MI355X VSS env.

Same command line (`--env-id sa|cma|dma --num-envs ... --num-steps ...`, ppo…:48-118), same
`Agent` (module order, orthogonal init, state-dict keys: ppo…:121-164), same rollout / GAE /
clipped-PPO update semantics (ppo…:231-365).  MI355X-first changes:

* the env is the fused HIP step (envs/wrappers.py), one launch per control step;
* data parallel over ranks (one process per GPU, `torch.distributed` = RCCL): each rank owns
  `--num-envs` environments (weak scaling; BASELINE config 5 = 8 x 65,536) and its own rollout
  storage; the only exchange is ONE all-reduce of a flat fp32 gradient buffer per minibatch
  (all parameter .grad tensors are views into it), between backward() and clip_grad_norm_
  (ppo…:352-353); approx_kl is averaged over ranks when it drives a decision;
* no per-element host-synchronising logging loop (ppo…:273-279): episode statistics are
  reduced on the device and read once per update;
* logging is optional (TensorBoard / W&B only if installed and requested).
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

# ROCm's graph packet capture.  In round 3 a captured 2,097,152-row minibatch replayed wrongly from its
# 9th launch on with it on (profiles/r03w_graph_probe2.log); in round 4 neither the same code (commit
# ea0c048) nor this tree reproduces that on any MLP / loss path, torch-only included
# (tools/graph_replay_probe.py, profiles/r04_graph_replay_probes.log), so the defect is not this
# repository's kernels and is not reproducible on demand.  The entry points (this script's __main__,
# bench.py, tools/time_to_score.py, tests/conftest.py) still start the runtime with it off
# (disable_graph_packet_capture); importing the module changes no environment variable, and every
# captured minibatch is guarded by MinibatchGraph's self-check against eager instead.
_PACKET_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"


def disable_graph_packet_capture() -> bool:
    """Entry points call this before anything initialises the GPU (the runtime reads the switch when it
    starts): sets DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 unless the environment already chose.  Returns
    whether the switch is now off."""
    if _PACKET_CAPTURE not in os.environ and not torch.cuda.is_initialized():
        os.environ[_PACKET_CAPTURE] = "0"
    return os.environ.get(_PACKET_CAPTURE) == "0"


import torch.nn as nn
import torch.optim as optim
from torch.distributions.normal import Normal

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from envs._gym import Box, ObservationWrapper  # noqa: E402
from vss_amd.loss import (N_ACT, adv_part_sum, minibatch_gather, minibatch_gather_parts, ppo_loss,  # noqa: E402
                          ppo_loss_direct, ppo_loss_fused_finish, randperm)
from vss_amd.update import (first_wgrad_ok, gemm_shape_ok, linear_tanh, linear_tanh_backward, linear_tanh_backward_mixed,  # noqa: E402
                            linear_tanh_loss_x6, linear_tanh_loss_x6_ok, linear_tanh_mixed, linear_tanh_out,
                            linear_tanh_out_mixed, linear_tanh_out_ok,
                            linear_tanh_out_x6, output_backward, output_backward_direct, output_backward_direct_ok,
                            output_backward_ok, sum_parts, weight_grad_mixed, weight_planes, x6_ok)


def strtobool(x: str) -> bool:
    v = str(x).lower()
    if v in ("y", "yes", "t", "true", "on", "1"):
        return True
    if v in ("n", "no", "f", "false", "off", "0"):
        return False
    raise ValueError(f"invalid truth value {x!r}")


def parse_args(argv=None):
    b = strtobool
    p = argparse.ArgumentParser()
    p.add_argument("--exp-name", type=str, default=os.path.basename(__file__).rstrip(".py"))
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--torch-deterministic", type=b, default=True, nargs="?", const=True)
    p.add_argument("--cuda", type=b, default=True, nargs="?", const=True)
    p.add_argument("--track", type=b, default=False, nargs="?", const=True)
    p.add_argument("--wandb-project-name", type=str, default="ppo-isaac-cleanrl")
    p.add_argument("--wandb-entity", type=str, default=None)
    p.add_argument("--capture-video", type=b, default=False, nargs="?", const=True)
    p.add_argument("--env-id", type=str, default="sa")
    p.add_argument("--total-timesteps", type=int, default=1000000000)
    p.add_argument("--learning-rate", type=float, default=0.001)
    p.add_argument("--num-envs", type=int, default=4095, help="environments per rank")
    p.add_argument("--num-steps", type=int, default=128)
    p.add_argument("--anneal-lr", type=b, default=False, nargs="?", const=True)
    p.add_argument("--adaptative-lr", type=b, default=False, nargs="?", const=True)
    p.add_argument("--gamma", type=float, default=0.99)
    p.add_argument("--gae-lambda", type=float, default=0.95)
    p.add_argument("--num-minibatches", type=int, default=4)
    p.add_argument("--update-epochs", type=int, default=8)
    p.add_argument("--norm-adv", type=b, default=True, nargs="?", const=True)
    p.add_argument("--clip-coef", type=float, default=0.2)
    p.add_argument("--clip-vloss", type=b, default=False, nargs="?", const=True)
    p.add_argument("--ent-coef", type=float, default=0.005)
    p.add_argument("--vf-coef", type=float, default=4)
    p.add_argument("--max-grad-norm", type=float, default=1.5)
    p.add_argument("--target-kl", type=float, default=None)
    p.add_argument("--threshold-kl", type=float, default=0.008)
    p.add_argument("--reward-scaler", type=float, default=1000)
    p.add_argument("--record-video-step-frequency", type=int, default=20000)
    p.add_argument("--test", type=b, default=False, nargs="?", const=True)
    # build additions
    p.add_argument("--save-path", type=str, default="runs")
    p.add_argument("--num-updates", type=int, default=None, help="override total_timesteps // batch")
    p.add_argument("--log", type=b, default=True, nargs="?", const=True)
    p.add_argument("--fused-policy", type=b, default=True, nargs="?", const=True,
                   help="rollout forward with the fused HIP MLP kernel (vss_policy_forward); "
                        "terminal values only for the fields that reset")
    p.add_argument("--evaluate", type=b, default=False, nargs="?", const=True,
                   help="after training, play matches vs the baseline teams (ppo…:380-461, no W&B)")
    p.add_argument("--eval-matches", type=int, default=10000, help="matches per baseline team")
    p.add_argument("--global-adv-norm", type=b, default=True, nargs="?", const=True,
                   help="with several ranks, normalise each minibatch's advantages with the mean / std "
                        "of the GLOBAL minibatch (all ranks' rows, one small all-reduce), as the "
                        "reference's single-process loop does (ppo…:324-326); off = per-rank statistics")
    p.add_argument("--amp", type=str, default="none", choices=["none", "bf16"],
                   help="bf16 autocast for the MLP GEMMs (off = the reference's fp32 numerics)")
    p.add_argument("--update-graph", type=b, default=True, nargs="?", const=True,
                   help="replay each minibatch's forward, losses and backward as one captured HIP graph "
                        "(MinibatchGraph; on a ROCm GPU with --amp none), eager otherwise")
    p.add_argument("--kernel-warmup", type=b, default=True, nargs="?", const=True,
                   help="before the train clock starts (ppo…:244), run one short update of the same loop on a "
                        "throwaway env and agent (16,384 envs x 8 steps), so the runtime loads the code objects of "
                        "the kernels the loop uses outside the clock (warmup_kernels; its time is kept in "
                        "args.kernel_warmup_s); the training itself is unchanged")
    args = p.parse_args(argv)
    args.batch_size = int(args.num_envs * args.num_steps)
    args.minibatch_size = int(args.batch_size // args.num_minibatches)
    return args


def layer_init(layer, std=np.sqrt(2), bias_const=0.0):
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def _mlp(n_in, n_out, last_std):
    return nn.Sequential(
        layer_init(nn.Linear(n_in, 256)), nn.Tanh(),
        layer_init(nn.Linear(256, 512)), nn.Tanh(),
        layer_init(nn.Linear(512, 512)), nn.Tanh(),
        layer_init(nn.Linear(512, 256)), nn.Tanh(),
        layer_init(nn.Linear(256, n_out), std=last_std),
    )


class Agent(nn.Module):
    """Separate actor / critic MLPs with a state-independent log-std (ppo…:127-164)."""

    def __init__(self, envs):
        super().__init__()
        n_obs = int(np.array(envs.single_observation_space.shape).prod())
        n_act = int(np.prod(envs.single_action_space.shape))
        self.critic = _mlp(n_obs, 1, 1.0)       # created first: same RNG consumption order
        self.actor_mean = _mlp(n_obs, n_act, 0.01)
        self.actor_logstd = nn.Parameter(torch.zeros(1, n_act))

    def get_value(self, x):
        return self.critic(x)

    def get_action_and_value(self, x, action=None):
        mean = self.actor_mean(x)
        std = torch.exp(self.actor_logstd.expand_as(mean))
        probs = Normal(mean, std)
        if action is None:
            action = probs.sample()
        return action, probs.log_prob(action).sum(1), probs.entropy().sum(1), self.critic(x)


# ---- the update's MLPs ---------------------------------------------------------------------------------
# The first layer's weight gradient dW = dY^T X reduces over all minibatch rows (2,097,152 at 65,536 envs)
# into a (256, 52) output; as one GEMM hipBLASLt runs it at ~1 TF.  Splitting the rows into SPLITK chunks
# (one batched GEMM + a sum) runs it at ~90 TF (tools/wgrad_bench.py); only the fp32 summation order differs.
SPLITK = 64
SPLITK_MIN_ROWS = 32768


def _split_k_wgrad(gz, x, out=None):
    rows = x.shape[0]
    if rows >= SPLITK_MIN_ROWS:
        # the rows in SPLITK equal chunks (one batched GEMM + a sum), the < SPLITK left over added
        main = rows // SPLITK * SPLITK
        dw = torch.sum(torch.bmm(gz[:main].reshape(SPLITK, main // SPLITK, gz.shape[1]).transpose(1, 2),
                                 x[:main].reshape(SPLITK, main // SPLITK, x.shape[1])), 0, out=out)
        return dw.addmm_(gz[main:].t(), x[main:]) if main < rows else dw
    return torch.mm(gz.t(), x, out=out)


class _TanhMLP(torch.autograd.Function):
    """The Agent's MLP (ppo…:104-111: (Linear, Tanh) x L + Linear) as ONE autograd node for the
    update.  Forward: each hidden layer is one GEMM launch with bias + tanh in its epilogue, the last
    one with the output layer folded in.  Backward: the output layer and the tanh below it in one
    streaming pass (vss_output_backward); every other hidden tanh by the input-gradient GEMM of the
    layer above with the tanh derivative and the bias-gradient column sums in its epilogue; weight
    gradients as split GEMMs over the rows.  UPDATE_GEMM "x6" (default) runs the GEMMs of the
    256/512-wide layers on the bf16 matrix cores in fp32 arithmetic (csrc/vss_gemm_x6.hip; whole
    256-row tiles, the ragged rest of a minibatch on the fp32-MFMA kernels), "fp32" on the fp32-MFMA
    kernels (csrc/vss_update.hip) only.  Inputs: x, W_0, b_0, ..., W_L, b_L."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        ctx.params = params  # the backward writes the FlatGrads-owned gradients in place (_grad_dst)
        hs = [x]
        rows = x.shape[0]
        x6 = x.is_cuda and UPDATE_GEMM == "x6"
        # the x6 layers' weight planes, forward (W) and backward (W^T), in one launch for the whole MLP
        pf, ctx.planes_b = _mlp_planes(ws, rows) if x6 else ({}, {})
        for layer, (w, b) in enumerate(zip(ws[:-2], bs[:-2])):
            if x6:
                hs.append(linear_tanh_mixed(hs[-1], w, b, planes=pf.get(layer)))
            else:
                hs.append(linear_tanh(hs[-1], w, b))
        if x6:
            # the last hidden layer and the output layer in one launch per row range (the whole 256-row
            # tiles through vss_linear_tanh_out_bf16x6, the rest through vss_linear_tanh + addmm)
            h, out = linear_tanh_out_mixed(hs[-1], ws[-2], bs[-2], ws[-1], bs[-1], planes=pf.get(len(ws) - 2))
            hs.append(h)
        elif x.is_cuda and linear_tanh_out_ok(rows, ws[-2].shape[1], ws[-2].shape[0], ws[-1].shape[0]):
            # the last hidden layer and the output layer in one launch (vss_linear_tanh_out)
            h, out = linear_tanh_out(hs[-1], ws[-2], bs[-2], ws[-1], bs[-1])
            hs.append(h)
        else:
            hs.append(linear_tanh(hs[-1], ws[-2], bs[-2]))
            out = torch.addmm(bs[-1], hs[-1], ws[-1].t())
        ctx.save_for_backward(*hs, *ws)
        return out

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        n = len(saved) // 2
        hs, ws = saved[:n], saved[n:]  # hs[l] = input of layer l (hs[0] = x), ws[l] = its weight
        grads = [None] * (2 * n)
        dst = [_grad_dst(p) if gout.is_cuda else None for p in ctx.params]
        # the split kernels' partial sums (weight gradients over row parts, bias column sums) reduced for
        # the whole MLP in one launch at the end (sum_parts), whether they go straight into FlatGrads or
        # back to autograd (the same kernels in the same order: the same bits either way)
        defer = [] if gout.is_cuda else None
        gz = gout.contiguous()  # pre-activation gradient of the current layer
        gb = torch.sum(gz, 0, out=dst[2 * n - 1])
        top = n - 1
        if n > 1 and output_backward_ok(gz.shape[1], hs[n - 1].shape[1]):
            # the output layer (1-6 columns): its weight gradient and the backward into the tanh layer
            # below in one streaming pass over that layer's output (vss_output_backward)
            grads[2 * n - 1] = gb
            gz, gb, grads[2 * n - 2] = output_backward(gz, ws[n - 1], hs[n - 1], out_db=dst[2 * n - 3],
                                                       out_dw=dst[2 * n - 2], defer=defer)
            top = n - 2
        gz = _backward_layers(hs, ws, ctx.planes_b, gz, gb, top, dst, grads, defer)
        if defer:
            sum_parts(defer)
        gx = gz.mm(ws[0]) if ctx.needs_input_grad[0] else None
        # the gradients already written into their parameters' .grad are not handed to autograd
        # (whose AccumulateGrad would add them to themselves)
        return (gx, *[None if d is not None else g for g, d in zip(grads, dst)])


def _backward_layers(hs, ws, planes_b, gz, gb, top: int, dst, grads, defer):
    """Layers top, top - 1, ..., 0 of an MLP backward (_TanhMLP.backward, direct_minibatch): gz = the
    pre-activation gradient of layer `top`, gb its bias gradient.  Each layer's weight gradient (x6 kernels
    or the split-K GEMM) into dst / grads, then the backward into the tanh layer below with the tanh
    derivative and the bias column sums in its epilogue (partial sums queued on `defer` when given).
    Returns the pre-activation gradient of layer 0."""
    n = len(ws)
    for layer in range(top, -1, -1):
        x6 = gz.is_cuda and UPDATE_GEMM == "x6"
        if x6 and ((hs[layer].shape[1] % 128 == 0 and gz.shape[1] % 256 == 0) or
                   (layer == 0 and first_wgrad_ok(256, gz.shape[1], hs[0].shape[1]))):
            # the hidden layers' and the first layer's weight gradients on the x6 kernels
            grads[2 * layer] = weight_grad_mixed(gz, hs[layer], out=dst[2 * layer], defer=defer)
        else:
            grads[2 * layer] = _split_k_wgrad(gz, hs[layer], out=dst[2 * layer])
        grads[2 * layer + 1] = gb
        if layer == 0:
            break
        w = ws[layer]
        if layer == n - 1 and gz.shape[1] % 4:
            # the output layer's few columns (1, 2 or 6): zero-padded to a multiple of 4, the
            # GEMM's contraction granule, so this backward is one fused pass as well
            pad = 4 - gz.shape[1] % 4
            gz, w = nn.functional.pad(gz, (0, pad)), nn.functional.pad(w, (0, 0, 0, pad))
        if x6:
            gz, gb = linear_tanh_backward_mixed(gz, w, hs[layer], out_db=dst[2 * layer - 1],
                                                planes=planes_b.get(layer) if layer < n - 1 else None, defer=defer)
        else:
            gz, gb = linear_tanh_backward(gz, w, hs[layer])
            if dst[2 * layer - 1] is not None:
                gb = dst[2 * layer - 1].copy_(gb)
    return gz


def _mlp_planes(ws, rows: int):
    """The bf16 planes of the hidden layers' weights the x6 GEMMs take (vss_weight_planes_bf16x6, one
    launch): {layer: planes of W} for the forwards of layers 1 .. L-2 and {layer: planes of W^T} for
    their backwards (layer 0's input width is the observation's, below the x6 shapes; layer L-1 is the
    output layer).  Valid for this minibatch: the weights change only at the optimizer step."""
    return _nets_planes([ws], rows)[0]


def _nets_planes(nets, rows: int):
    """_mlp_planes for several MLPs (nets = [their weight lists]) in one launch while the jobs fit it."""
    if rows < 256:
        return [({}, {}) for _ in nets]
    jobs = []
    for q, ws in enumerate(nets):
        for layer in range(1, len(ws) - 1):
            n, k = ws[layer].shape
            if x6_ok(256, k, n):
                jobs.append((q, layer, False))
            if x6_ok(256, n, k):
                jobs.append((q, layer, True))
    out = [({}, {}) for _ in nets]
    for j0 in range(0, len(jobs), 16):
        chunk = jobs[j0:j0 + 16]
        planes = weight_planes([(nets[q][layer], tr) for q, layer, tr in chunk])
        for (q, layer, tr), p in zip(chunk, planes):
            out[q][1 if tr else 0][layer] = p
    return out


# the fused path's GEMM arithmetic: "x6" (default) = fp32 products on the bf16 matrix cores from an
# exact 3-way bf16 split of every operand (csrc/vss_gemm_x6.hip; error vs fp64 at or below the fp32
# GEMMs', tests/test_gemm_x6.py), where the shapes are exact; "fp32" = the fp32-MFMA kernels only.
# (The round-4 A/B switches VSS_UPDATE_MLP=split, VSS_OUTPUT_FWD/BWD=0 and VSS_WEIGHT_PLANES=0, each
# strictly slower, are retired from the product: tools/ab_switches_r04.patch re-adds them for A/B runs.)
UPDATE_GEMM = os.environ.get("VSS_UPDATE_GEMM", "x6")
# direct_minibatch's loss folded into the last hidden layer's x6 launch (vss_linear_tanh_loss_bf16x6) where
# the output layers allow it; "0" keeps the separate output-layer / loss / output-backward launches
FUSED_LOSS = os.environ.get("VSS_FUSED_LOSS", "1") != "0"
# the epochs' permutations on a ROCm device from vss_randperm (one seed per epoch from the update's
# generator); VSS_RANDPERM=torch keeps torch.randperm
RANDPERM_HIP = os.environ.get("VSS_RANDPERM", "hip") != "torch"


def _fused_mlp_ok(seq: nn.Sequential) -> bool:
    mods = list(seq)
    if len(mods) < 3 or len(mods) % 2 == 0:
        return False
    lins, acts = mods[0::2], mods[1::2]
    if not all(type(m) is nn.Linear and m.bias is not None for m in lins) or \
            not all(isinstance(a, nn.Tanh) for a in acts):
        return False
    return all(gemm_shape_ok(m.in_features, m.out_features) for m in lins[:-1]) and \
        all(gemm_shape_ok((m.out_features + 3) // 4 * 4, m.in_features) for m in lins[1:])


def _mlp_forward(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """The update's MLP: _TanhMLP for the Agent's (Linear, Tanh) x L + Linear stacks in fp32, the module
    itself (torch autograd) for anything else."""
    if x.dtype == torch.float32 and _fused_mlp_ok(seq):
        params = [t for m in list(seq)[0::2] for t in (m.weight, m.bias)]
        return _TanhMLP.apply(x, *params)
    return seq(x)


def get_action_and_value_update(agent: "Agent", x, action):
    """Agent.get_action_and_value (ppo…:157-164) on the same parameters, for the PPO update: the
    same function (forward within fp32 rounding: fused GEMM summation order and a few-ulp tanh),
    the MLPs through _TanhMLP."""
    mean = _mlp_forward(agent.actor_mean, x)
    std = torch.exp(agent.actor_logstd.expand_as(mean))
    # no argument validation: its finiteness check is a host sync per minibatch, which a captured
    # minibatch (MinibatchGraph) cannot hold; the loss values are the same
    probs = Normal(mean, std, validate_args=False)
    return action, probs.log_prob(action).sum(1), probs.entropy().sum(1), _mlp_forward(agent.critic, x)


class ExtractObsWrapper(ObservationWrapper):
    def observation(self, obs):
        return obs["obs"]


_DIRECT_GRADS = [False]  # set by FlatGrads.zeroed_backward() around the update's loss.backward()


def _grad_dst(p: torch.Tensor):
    """The .grad of a FlatGrads-owned parameter, which _TanhMLP's backward writes directly inside
    FlatGrads.zeroed_backward(): the buffer was zeroed just before and each parameter receives exactly
    one gradient per backward, so writing it equals autograd's accumulation into zero -- without one add
    kernel per parameter.  None anywhere else (plain autograd: torch.autograd.grad, other callers)."""
    g = p.grad
    if _DIRECT_GRADS[0] and getattr(p, "_vss_flat_grad", False) and g is not None and g.is_cuda \
            and g.dtype == torch.float32:
        return g
    return None


class FlatGrads:
    """All parameter gradients as views of ONE contiguous fp32 buffer, so the data-parallel
    exchange is a single all-reduce (4.3 MB for the SA agent) with no pack/unpack copies.  The MLPs'
    backward (_TanhMLP) writes their gradients straight into these views (_grad_dst).  With
    flat_params the parameters themselves become views of one buffer as well (same order), which
    FlatAdam steps in one launch."""

    ALIGN = 64  # floats: every tensor starts 256-B aligned (the HIP entries take 16-B aligned buffers)

    def __init__(self, module: nn.Module, flat_params: bool = False):
        self.params = [p for p in module.parameters() if p.requires_grad]
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off = -(-(off + p.numel()) // self.ALIGN) * self.ALIGN
        dev = self.params[0].device
        # the gaps between tensors stay zero in both buffers (zero gradients leave them unchanged)
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        self.flat_p = torch.zeros(off, device=dev, dtype=torch.float32) if flat_params else None
        self.optimizer = None  # a FlatAdam stepping these buffers (clip_norm_ then defers to it)
        for p, o in zip(self.params, offs):
            p.grad = self.flat[o:o + p.numel()].view_as(p)
            p._vss_flat_grad = True
            if flat_params:
                if p.dtype != torch.float32:
                    raise ValueError("flat_params: fp32 parameters only")
                view = self.flat_p[o:o + p.numel()].view_as(p)
                view.copy_(p.detach())
                p.data = view

    def zero(self):
        self.flat.zero_()

    def zeroed_backward(self, loss: torch.Tensor):
        """zero() then loss.backward() (ppo…:351-352), the MLPs' gradients written in place (_grad_dst)."""
        self.zero()
        _DIRECT_GRADS[0] = True
        try:
            loss.backward()
        finally:
            _DIRECT_GRADS[0] = False

    def all_reduce_mean(self, world: int):
        if world > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            self.flat.mul_(1.0 / world)

    def clip_norm_(self, max_norm: float) -> torch.Tensor:
        """nn.utils.clip_grad_norm_(agent.parameters(), max_norm) (ppo…:353) on the flat buffer: the L2
        norm of all the gradients (one reduction instead of one per tensor and a norm of the norms), the
        same coefficient max_norm / (norm + 1e-6) clamped to 1, one in-place scale.  Returns the norm.
        With a FlatAdam attached the scale is applied inside its next step() (the norm's partial sums are
        taken here, vss_grad_sq_partials; the returned tensor holds the norm once that step has run)."""
        if self.optimizer is not None:
            return self.optimizer.defer_clip(max_norm)
        total = torch.linalg.vector_norm(self.flat)
        self.flat.mul_(torch.clamp(max_norm / (total + 1e-6), max=1.0))
        return total


class FlatAdam(torch.optim.Optimizer):
    """optim.Adam(agent.parameters(), lr, eps=1e-5) (ppo…:166, step at ppo…:354) over FlatGrads' flat
    parameter and gradient buffers: one launch (vss_adam_step_clipped) per step, which also applies the
    clip_grad_norm_ (ppo…:353) requested through FlatGrads.clip_norm_ just before -- instead of torch's
    norm chain and multi-tensor Adam (~8 launches, ~130 us per minibatch at the reference's 4,095 envs).
    Same update rule, in torch's fused-Adam arithmetic (tests/test_ppo.py); param_groups[0]["lr"] is read
    at every step, so --anneal-lr / --adaptative-lr act on it as on torch's Adam."""

    def __init__(self, flat: FlatGrads, lr: float, betas=(0.9, 0.999), eps: float = 1e-5):
        if flat.flat_p is None or not flat.flat.is_cuda:
            raise ValueError("FlatAdam: a FlatGrads with flat_params=True on a ROCm device")
        super().__init__(flat.params, dict(lr=lr, betas=betas, eps=eps))
        from vss_amd import _native as N
        self._N = N
        self.flat = flat
        flat.optimizer = self
        n = flat.flat.numel()
        self.exp_avg = torch.zeros_like(flat.flat_p)
        self.exp_avg_sq = torch.zeros_like(flat.flat_p)
        self.steps = 0
        self.nparts = int(N.load().vss_grad_sq_partials_count(n))
        self.partial = torch.zeros(self.nparts, device=flat.flat.device)
        self.norm = torch.zeros(1, device=flat.flat.device)
        self._max_norm = 0.0

    def zero_grad(self, set_to_none: bool = True):
        """Zero the flat gradient buffer (the .grad tensors are views of it and stay in place)."""
        self.flat.zero()

    def defer_clip(self, max_norm: float) -> torch.Tensor:
        """Take the norm's partial sums of the current gradients now; the next step() applies the clip."""
        N = self._N
        N.check(N.load().vss_grad_sq_partials(N.stream_of(self.flat.flat.device), self.flat.flat.numel(),
                                              self.flat.flat.data_ptr(), self.partial.data_ptr()),
                "vss_grad_sq_partials")
        self._max_norm = float(max_norm)
        return self.norm

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise ValueError("FlatAdam.step: no closure")
        N = self._N
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        self.steps += 1
        f = self.flat
        N.check(N.load().vss_adam_step_clipped(
            N.stream_of(f.flat.device), f.flat.numel(), self.nparts, self.partial.data_ptr(), self._max_norm,
            float(g["lr"]), float(b1), float(b2), float(g["eps"]), self.steps, f.flat.data_ptr(), f.flat_p.data_ptr(),
            self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.norm.data_ptr()), "vss_adam_step_clipped")
        self._max_norm = 0.0  # a clip applies to the step right after it only


class _NullWriter:
    def add_scalar(self, *a, **k):
        pass

    def add_text(self, *a, **k):
        pass

    def close(self):
        pass


class _CsvWriter:
    """The SummaryWriter calls the loop makes, appended to `<run>/scalars.csv` (tag,value,step)
    when TensorBoard is not installed, so the learning curves are kept either way."""

    def __init__(self, path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        self._f = open(path, "w")
        self._f.write("tag,value,step\n")

    def add_scalar(self, tag, value, step):
        self._f.write(f"{tag},{float(value)!r},{int(step)}\n")

    def add_text(self, *a, **k):
        pass

    def close(self):
        self._f.close()


def make_writer(args, run_name, rank):
    if rank != 0 or not args.log:
        return _NullWriter()
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(f"{args.save_path}/{run_name}")
    except ImportError:  # tensorboard not installed
        return _CsvWriter(f"{args.save_path}/{run_name}/scalars.csv")


EP_KEYS = ("goal", "grad", "move", "energy", "return")  # info['r'] keys (envs/wrappers.py:74-80)


def first_done_stats(done: torch.Tensor, info: dict) -> torch.Tensor:
    """[any done, goal, grad, move, energy, return, length] of the FIRST env with done set — what
    ppo…:273-279 logs by looping over the envs on the host — as one device tensor, no sync."""
    d = done.float()
    idx = torch.argmax(d)  # index of the first maximum
    return torch.stack([d.max()] + [info["r"][k][idx].float() for k in EP_KEYS] + [info["l"][idx].float()])


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


def compute_gae(rewards, values, next_values, next_dones, next_timeouts, gamma, lam):
    """Timeout-aware GAE of ppo…:282-296 (terminal-obs bootstrap, reversed scan over T)."""
    T = rewards.shape[0]
    advantages = torch.zeros_like(rewards)
    next_non_terminal = 1.0 - next_dones.logical_and(next_timeouts.logical_not()).float()
    lastgaelam = torch.zeros_like(rewards[0])
    for t in reversed(range(T)):
        delta = rewards[t] + gamma * next_values[t] * next_non_terminal[t] - values[t]
        lastgaelam = delta + gamma * lam * (1.0 - next_dones[t]) * lastgaelam
        advantages[t] = lastgaelam
    return advantages, advantages + values


def autocast(args, device):
    """bf16 autocast for the MLP GEMMs when --amp bf16 (fp32 master weights, fp32 losses)."""
    enabled = getattr(args, "amp", "none") == "bf16" and torch.device(device).type == "cuda"
    return torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=enabled)


def normalize_advantages(mb_adv: torch.Tensor, world: int = 1, global_stats: bool = True) -> torch.Tensor:
    """(a - mean) / (std + 1e-8) of ppo…:325-326.  One rank (or per-rank statistics): torch's own
    mean / unbiased std, exactly the reference's expression.  Several ranks with global_stats:
    the mean and unbiased std of the union of every rank's minibatch rows -- the minibatch the
    reference would have drawn in one process -- from one all-reduce of (sum, sum of squares,
    count) in float64."""
    if world == 1 or not global_stats:
        return (mb_adv - mb_adv.mean()) / (mb_adv.std() + 1e-8)
    a = mb_adv.double()
    s = torch.stack([a.sum(), (a * a).sum(), torch.tensor(float(a.numel()), dtype=torch.float64, device=a.device)])
    dist.all_reduce(s)
    n = s[2]
    mean = s[0] / n
    std = ((s[1] - n * mean * mean) / (n - 1)).clamp(min=0).sqrt()
    return (mb_adv - mean.float()) / (std.float() + 1e-8)


def annealed_lr(update: int, num_updates: int, lr0: float) -> float:
    """--anneal-lr (ppo…:251-253): linear decay from lr0 at update 1 to lr0 / num_updates at the last."""
    frac = 1.0 - (update - 1.0) / num_updates
    return frac * lr0


def adapted_lr(lr: float, approx_kl: float, threshold_kl: float) -> float:
    """--adaptative-lr (ppo…:356-361), after every minibatch: /1.5 (floor 1e-6) when the KL estimate
    exceeds 2 x threshold, x1.5 (cap 1e-2) when it is below threshold / 2, else unchanged."""
    if approx_kl > 2.0 * threshold_kl:
        return max(lr / 1.5, 1e-6)
    if approx_kl < 0.5 * threshold_kl:
        return min(lr * 1.5, 1e-2)
    return lr


def value_loss(newvalue, mb_returns, mb_values, clip_coef: float, clip_vloss: bool):
    """The value loss of ppo…:335-346: 0.5 mean (v - R)^2, or with --clip-vloss the elementwise max
    of that and the loss of v clipped to within clip_coef of the rollout's value."""
    if clip_vloss:
        v_unclipped = (newvalue - mb_returns) ** 2
        v_clipped = mb_values + torch.clamp(newvalue - mb_values, -clip_coef, clip_coef)
        return 0.5 * torch.max(v_unclipped, (v_clipped - mb_returns) ** 2).mean()
    return 0.5 * ((newvalue - mb_returns) ** 2).mean()


# the update's minibatch rows are padded to a multiple of this (MLP_ROW_PAD) on the GPU, so that every
# hidden-layer GEMM runs on whole x6 tiles: at 4,095 envs a 131,040-row minibatch otherwise leaves
# 224-row tails that hipBLASLt runs on one or two workgroups (43-110 us each, ~21 ms per update)
MLP_ROW_PAD = 256
# MinibatchGraph re-runs replays 12, 48, 192, ... (GRAPH_CHECK_REPLAY x GRAPH_CHECK_FACTOR^m) eagerly and
# compares each with its replay bit for bit: round 3's packet-capture failure began at the 9th replay
# (profiles/r03w_graph_probe2.log), and a later onset is caught at the next check; the checks cost one eager
# minibatch each, O(log replays) per run
GRAPH_CHECK_REPLAY = 12
GRAPH_CHECK_FACTOR = 4


def graph_check_due(replays: int) -> bool:
    """Whether replay number `replays` (1-based) of a MinibatchGraph is re-run eagerly and compared."""
    r = GRAPH_CHECK_REPLAY
    while r < replays:
        r *= GRAPH_CHECK_FACTOR
    return r == replays


def minibatch_losses(agent, args, obs, actions, logprobs, adv, returns, values):
    """The clipped PPO losses of ppo…:318-349 on one minibatch (adv already normalised when
    --norm-adv): (loss, (pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac)).
    obs / actions may carry padding rows beyond the minibatch's len(logprobs) (copies of its first
    rows): the networks run over them, the losses do not see them, so their gradient is zero."""
    if getattr(args, "amp", "none") == "none":
        # the networks (_TanhMLP on the GPU) ...
        mean = _mlp_forward(agent.actor_mean, obs)
        value = _mlp_forward(agent.critic, obs)
    else:  # --amp bf16: the networks under autocast, the loss in fp32
        with autocast(args, obs.device):
            mean, value = agent.actor_mean(obs), agent.critic(obs)
        mean, value = mean.float(), value.float()
    # ... then the loss and its gradients into the networks' outputs as one autograd node (vss_ppo_loss:
    # two launches on the GPU instead of ~100; the reference's expressions on the CPU)
    return ppo_loss(mean, agent.actor_logstd, value, actions, logprobs, adv, returns, values, args.clip_coef,
                    args.ent_coef, args.vf_coef, args.clip_vloss)


# ---- the update's minibatch without autograd (round 5) --------------------------------------------------
# On a ROCm device the minibatch's forward, loss and backward are ONE fixed sequence of this repository's
# launches (direct_minibatch), not an autograd graph: the output layers' epilogue parts go straight into
# the loss (vss_ppo_loss_direct: no sum / bias-add launches, the advantage normalisation and the output
# biases' gradients inside it), the loss's row gradients straight into the output layers' backward
# (vss_output_backward_direct: no padded copies, no autograd scaling by the loss's incoming gradient of 1),
# and every gradient is written into its FlatGrads view (no zeroing, no AccumulateGrad); the rows come from
# one gather launch (vss_minibatch_gather) instead of six gathers, a cat and the mean / std chain.  The
# kernels are those of the autograd path (_TanhMLP); the results differ from it by summation order only
# (tests/test_ppo.py::test_direct_minibatch_matches_autograd_path_gpu).

def _mlp_wb(seq: nn.Sequential):
    lins = list(seq)[0::2]
    return [m.weight for m in lins], [m.bias for m in lins]


def direct_minibatch_ok(agent, args, flat) -> bool:
    """Whether the update's minibatches run as direct_minibatch: x6 GEMMs, fp32 (no --amp), both MLPs the
    Agent's (Linear, Tanh) x L + Linear stacks with a 256-wide last hidden layer on the x6 shapes (its
    output layer's parts feed the loss: 1, 2 or 6 outputs, the actor's n_act in the loss's set, the critic
    one value), and every parameter's .grad a FlatGrads view on the GPU."""
    if flat is None or UPDATE_GEMM != "x6" or getattr(args, "amp", "none") != "none":
        return False
    for seq, outs in ((agent.actor_mean, N_ACT), (agent.critic, (1,))):
        if not _fused_mlp_ok(seq):
            return False
        ws, _ = _mlp_wb(seq)
        if len(ws) < 3:
            return False
        (n, k), k_out = ws[-2].shape, ws[-1].shape[0]
        if not (x6_ok(256, k, n) and n == 256 and k_out in (1, 2, 6) and k_out in outs
                and output_backward_direct_ok(k_out, n)):
            return False
    owned = {id(p) for p in flat.params}
    return all(id(p) in owned and getattr(p, "_vss_flat_grad", False) and p.grad is not None and p.grad.is_cuda
               and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
               for p in agent.parameters() if p.requires_grad)


def _fused_loss_ok(agent, rows_pad: int) -> bool:
    """Whether direct_minibatch folds the loss into the last hidden layers' launches: the actor's 1 or 2
    outputs, the critic's value (direct_minibatch_ok's networks otherwise)."""
    for seq in (agent.actor_mean, agent.critic):
        ws, _ = _mlp_wb(seq)
        (n, k), k_out = ws[-2].shape, ws[-1].shape[0]
        if not linear_tanh_loss_x6_ok(rows_pad, k, n, k_out):
            return False
    return _mlp_wb(agent.critic)[0][-1].shape[0] == 1


def direct_minibatch(agent, args, obs, act, logp, adv, adv_part, adv_count, ret, val):
    """One update minibatch (ppo…:331-352: the networks, the clipped losses, loss.backward() into the
    zeroed gradients) as a fixed launch sequence writing every gradient into its FlatGrads view.  obs / act
    (rows_pad rows, the padding repeating the minibatch), logp / adv / ret / val (rows); adv RAW, normalised
    inside the loss from adv_part / adv_count (vss_ppo_loss_direct; None: as given).  Returns (loss,
    (pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac))."""
    (pfa, pba), (pfc, pbc) = _nets_planes([_mlp_wb(agent.actor_mean)[0], _mlp_wb(agent.critic)[0]], obs.shape[0])
    planes = {id(agent.actor_mean): (pfa, pba), id(agent.critic): (pfc, pbc)}

    def forward(seq):
        ws, bs = _mlp_wb(seq)
        pf, pb = planes[id(seq)]
        hs = [obs]
        for layer in range(len(ws) - 2):
            hs.append(linear_tanh_mixed(hs[-1], ws[layer], bs[layer], planes=pf.get(layer)))
        y, parts = linear_tanh_out_x6(hs[-1], ws[-2], bs[-2], ws[-1], bs[-1], planes=pf.get(len(ws) - 2), parts=True)
        hs.append(y)
        return hs, ws, bs, parts, pb, [t.grad for w, b in zip(ws, bs) for t in (w, b)]

    def backward(net, g, defer):
        hs, ws, _, _, pb, d = net
        n = len(ws)
        gz, gb, _ = output_backward_direct(g, ws[-1], hs[-1], out_db=d[2 * n - 3], out_dw=d[2 * n - 2], defer=defer)
        _backward_layers(hs, ws, pb, gz, gb, n - 2, d, [None] * (2 * n), defer)

    def fused(seq, is_actor, defer):
        # the hidden layers below the last, then the last hidden layer + output layer + this network's loss
        # terms + the output layer's backward in one launch
        ws, bs = _mlp_wb(seq)
        pf, pb = planes[id(seq)]
        n = len(ws)
        d = [t.grad for w, b in zip(ws, bs) for t in (w, b)]
        hs = [obs]
        for layer in range(n - 2):
            hs.append(linear_tanh_mixed(hs[-1], ws[layer], bs[layer], planes=pf.get(layer)))
        role = dict(act=act, logp=logp, adv=adv, adv_part=adv_part, adv_count=adv_count,
                    logstd=agent.actor_logstd) if is_actor else dict(ret=ret, val=val)
        gz, gb, _, st = linear_tanh_loss_x6(hs[-1], ws[-2], bs[-2], ws[-1], bs[-1], logp.shape[0], is_actor,
                                            planes=pf.get(n - 2), clip_coef=args.clip_coef, vf_coef=args.vf_coef,
                                            clip_vloss=args.clip_vloss, out_db=d[2 * n - 3], out_dw=d[2 * n - 2],
                                            defer=defer, **role)
        return (hs, ws, pb, gz, gb, n, d), st

    # one stream: the critic's launches on a second stream beside the actor's were measured and not kept
    # (4,095 envs: 0.153 vs 0.154 s per update; 65,536: 2.33 vs 2.30 s -- concurrent GEMMs contend)
    if FUSED_LOSS and _fused_loss_ok(agent, obs.shape[0]):
        with torch.no_grad():
            defer = []
            a_net, a_st = fused(agent.actor_mean, True, defer)
            c_net, c_st = fused(agent.critic, False, defer)
            loss, stats = ppo_loss_fused_finish(a_st, c_st, logp.shape[0], agent.actor_logstd, args.ent_coef,
                                                args.vf_coef, agent.actor_logstd.grad, a_net[6][-1], c_net[6][-1])
            for hs, ws, pb, gz, gb, n, d in (a_net, c_net):
                _backward_layers(hs, ws, pb, gz, gb, n - 2, d, [None] * (2 * n), defer)
            sum_parts(defer)
        return loss, tuple(stats[i] for i in range(6))
    with torch.no_grad():
        actor, critic = forward(agent.actor_mean), forward(agent.critic)
        (_, _, ba, pa, _, da), (_, _, bc, pc, _, dc) = actor, critic
        g_mean, g_value, loss, stats = ppo_loss_direct(
            pa, ba[-1], pc, bc[-1], agent.actor_logstd, act, logp, adv, adv_part, adv_count, ret, val, args.clip_coef,
            args.ent_coef, args.vf_coef, args.clip_vloss, agent.actor_logstd.grad, da[-1], dc[-1])
        defer = []
        backward(actor, g_mean, defer)
        backward(critic, g_value, defer)
        sum_parts(defer)  # every weight / bias gradient's partial sums, both MLPs, one launch
    return loss, tuple(stats[i] for i in range(6))


class DirectRows:
    """One minibatch's rows for direct_minibatch: obs / act (rows_pad), logp / adv / ret / val (mb) and the
    advantages' (sum, sum of squares) parts, filled by gather() (vss_minibatch_gather, one launch)."""

    def __init__(self, mb: int, rows_pad: int, obs_w: int, act_w: int, device):
        z = lambda *shape, dtype=torch.float32: torch.zeros(shape, device=device, dtype=dtype)  # noqa: E731
        self.obs, self.act = z(rows_pad, obs_w), z(rows_pad, act_w)
        self.logp, self.adv, self.ret, self.val = z(mb), z(mb), z(mb), z(mb)
        self.adv_part = z(minibatch_gather_parts(mb), 2, dtype=torch.float64)
        self.adv_glob = z(1, 2, dtype=torch.float64)

    def gather(self, inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, norm_adv: bool,
               world: int = 1, global_stats: bool = True):
        """The rows of inds; returns the (adv_part, adv_count) the loss normalises with: this minibatch's
        parts, or with several ranks and global_stats their sum all-reduced over the ranks (the union's
        statistics, as normalize_advantages), or (None, 0) without --norm-adv."""
        minibatch_gather(inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, self.obs, self.act,
                         self.logp, self.adv, self.ret, self.val, self.adv_part)
        mb = inds.numel()
        if not norm_adv:
            return None, 0.0
        if world > 1 and global_stats:
            adv_part_sum(self.adv_part, self.adv_glob)
            dist.all_reduce(self.adv_glob)
            return self.adv_glob, float(mb * world)
        return self.adv_part, float(mb)


class MinibatchGraph:
    """One minibatch's forward, losses and backward (into FlatGrads) captured once as a HIP graph and
    replayed for every minibatch: ~300 launches (the MLP GEMMs, the loss and its autograd ops, the
    gradient zeroing) become one graph launch.  At the reference's 4,095 envs the update is launch-
    bound -- 131,040-row minibatches, 12,000 launches per update, the GPU idle ~23 % of it
    (profiles/r03w_trace_summary.txt).  The gathers into the static inputs, the advantage
    normalisation (with its all-reduce when world > 1), the gradient all-reduce, clipping and the
    Adam step run eagerly around the replay, so the optimizer is torch's own (host-side bias
    corrections) and the learning-rate schedules apply unchanged.  The kernels and their order are
    the eager path's, so the results are the same bits (tests/test_ppo.py)."""

    def __init__(self, agent, flat, args, mb, obs_dim, act_dim, device):
        self.agent, self.flat, self.args = agent, flat, args
        z = lambda *shape: torch.zeros(shape, device=device)  # noqa: E731
        mb_pad = mb + padding_rows(mb, device)
        # direct_minibatch (no autograd) when the networks allow it, with its one-launch gather
        self.direct = direct_minibatch_ok(agent, args, flat)
        if self.direct:
            self.rows = DirectRows(mb, mb_pad, int(np.prod(obs_dim)), int(np.prod(act_dim)), device)
            self.obs, self.act, self.logp = self.rows.obs, self.rows.act, self.rows.logp
            self.adv_src = None  # the (adv_part, adv_count) the captured loss reads
        else:
            self.obs, self.act = z(mb_pad, *obs_dim), z(mb_pad, *act_dim)
            self.logp, self.adv, self.ret, self.val = z(mb), z(mb), z(mb), z(mb)
        self.graph = None
        self.warm = False
        self.out = None
        self.replays = 0
        self.failed = False  # a self-check found the replay differing from eager: eager from then on

    def _body(self):
        if self.direct:
            r = self.rows
            _, st = direct_minibatch(self.agent, self.args, r.obs, r.act, r.logp, r.adv, *self.adv_src, r.ret, r.val)
            return st
        loss, st = minibatch_losses(self.agent, self.args, self.obs, self.act, self.logp, self.adv, self.ret,
                                    self.val)
        self.flat.zeroed_backward(loss)
        # detached: no autograd graph (and no AccumulateGrad node bound to this stream) outlives the step
        return tuple(t.detach() for t in st)

    def _capture(self):
        # the first minibatch ran eagerly (library handles, workspaces, lazy initialisation); release the
        # eager pool's cached blocks only when the device could not hold a second copy of them beside
        # the graph's private pool (a minibatch of DMA config 4 holds ~100 GB of activations and gradients)
        torch.cuda.synchronize()
        free, _ = torch.cuda.mem_get_info()
        if free < 1.25 * (torch.cuda.memory_reserved() - torch.cuda.memory_allocated()):
            torch.cuda.empty_cache()
        g = torch.cuda.CUDAGraph()
        # thread_local: with several ranks, RCCL's and the process group's own threads keep querying
        # their streams and events while this thread captures (no collective is captured)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.out = self._body()
        self.graph = g

    def run(self, inds, inds_pad, b_obs, b_actions, b_logprobs, mb_adv, b_returns, b_values):
        if inds.numel() != self.logp.numel() or inds_pad.numel() != self.obs.shape[0] or \
                b_obs.shape[1:] != self.obs.shape[1:] or b_actions.shape[1:] != self.act.shape[1:]:
            raise ValueError(f"MinibatchGraph: minibatch {inds.numel()} (+{inds_pad.numel() - inds.numel()} padding) "
                             f"x {tuple(b_obs.shape[1:])} does not match the captured "
                             f"{self.logp.numel()} (+{self.obs.shape[0] - self.logp.numel()}) x {tuple(self.obs.shape[1:])}")
        torch.index_select(b_obs, 0, inds_pad, out=self.obs)
        torch.index_select(b_actions, 0, inds_pad, out=self.act)
        torch.index_select(b_logprobs, 0, inds, out=self.logp)
        torch.index_select(b_returns, 0, inds, out=self.ret)
        torch.index_select(b_values, 0, inds, out=self.val)
        self.adv.copy_(mb_adv)
        return self._step()

    def run_direct(self, inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, world: int = 1):
        """The direct flow: the minibatch's rows gathered into the static buffers in one launch (RAW
        advantages; the loss normalises them), then the step (replay / eager / capture as run())."""
        if inds.numel() != self.logp.numel() or b_obs[0].numel() != self.obs.shape[1] or \
                b_actions[0].numel() != self.act.shape[1]:
            raise ValueError(f"MinibatchGraph: minibatch {inds.numel()} x {tuple(b_obs.shape[1:])} does not match the "
                             f"captured {self.logp.numel()} x {self.obs.shape[1]}")
        src = self.rows.gather(inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values,
                               self.args.norm_adv, world, getattr(self.args, "global_adv_norm", True))
        if self.graph is not None and (src[0] is not self.adv_src[0] or src[1] != self.adv_src[1]):
            raise ValueError("MinibatchGraph: the advantage normalisation changed after the capture")
        self.adv_src = src
        return self._step()

    def _step(self):
        if self.failed:
            return self._body()
        if self.graph is None:
            if not self.warm:  # the first minibatch: eager, real work
                self.warm = True
                return self._body()
            self._capture()
        self.graph.replay()
        self.replays += 1
        if graph_check_due(self.replays):
            return self._check()
        return self.out

    def _check(self):
        """Self-check of one replay: the same minibatch again, eagerly, on the same static inputs; the
        replay's statistics and gradients must equal the eager ones bit for bit (the kernels and their
        order are the same).  On a difference the graph is dropped and every later minibatch runs
        eagerly (the eager result, already in FlatGrads, is this minibatch's)."""
        got = [t.clone() for t in self.out] + [self.flat.flat.clone()]
        want = list(self._body())
        same = all(torch.equal(a, b) for a, b in zip(got, want + [self.flat.flat]))
        if same:
            return self.out
        import warnings
        warnings.warn(f"MinibatchGraph: replay {self.replays} differs from the eager minibatch; the update runs "
                      f"eagerly from here on (DEBUG_CLR_GRAPH_PACKET_CAPTURE="
                      f"{os.environ.get(_PACKET_CAPTURE, '<unset>')})", RuntimeWarning)
        self.failed, self.graph = True, None
        return tuple(want)


def padding_rows(mb: int, device) -> int:
    """Rows the update adds to a minibatch of mb rows (MLP_ROW_PAD on a ROCm GPU, none on the CPU)."""
    return (-mb) % MLP_ROW_PAD if torch.device(device).type == "cuda" else 0


_WARNED_PACKET_CAPTURE = [False]


def make_minibatch_graph(agent, flat, args, batch, obs_dim, act_dim, device):
    """MinibatchGraph when --update-graph applies (ROCm GPU, fp32, equal minibatches, and the runtime
    started with graph packet capture off), else None: the update then runs eagerly."""
    mb = batch // args.num_minibatches
    if not getattr(args, "update_graph", False) or torch.device(device).type != "cuda" or \
            getattr(args, "amp", "none") != "none" or batch % mb:
        return None
    if os.environ.get(_PACKET_CAPTURE) != "0":
        # a caller that initialised the GPU before disable_graph_packet_capture() (or chose packet capture
        # on): no capture -- round 3's corrupted replays ran in that mode (profiles/r03w_graph_probe2.log)
        if not _WARNED_PACKET_CAPTURE[0]:
            import warnings
            warnings.warn(f"{_PACKET_CAPTURE}={os.environ.get(_PACKET_CAPTURE, '<unset>')}: the runtime started "
                          "with graph packet capture on, so the update minibatches run eagerly (call "
                          "disable_graph_packet_capture() before anything initialises the GPU)", RuntimeWarning)
            _WARNED_PACKET_CAPTURE[0] = True
        return None
    return MinibatchGraph(agent, flat, args, mb, obs_dim, act_dim, device)


_SIDE_STREAMS = {}


class EpochPermutations:
    """The update's per-epoch minibatch permutations (ppo…:309, torch.randperm(batch) from `gen`, in epoch
    order; on a ROCm device vss_randperm from one seed per epoch drawn from `gen`).  On a ROCm device with
    ahead=True (no --target-kl early stop, so every epoch's permutation is drawn), epoch e + 1's is drawn
    on a side stream while epoch e's minibatches run, overlapping the GEMMs instead of preceding the
    epoch's first minibatch.  The generator is consumed in the same order: the same permutations."""

    def __init__(self, batch: int, device, gen, epochs: int, ahead: bool = True):
        self.batch, self.device, self.gen, self.left = batch, torch.device(device), gen, epochs
        self.side = None
        if ahead and self.device.type == "cuda":
            key = self.device.index if self.device.index is not None else torch.cuda.current_device()
            self.side = _SIDE_STREAMS.setdefault(key, torch.cuda.Stream(device=self.device))
        self.pending = None

    def _perm(self):
        if self.device.type != "cuda" or not RANDPERM_HIP or self.batch >= 2 ** 31:
            return torch.randperm(self.batch, device=self.device, generator=self.gen)
        # ROCm: vss_randperm from one seed drawn from gen (the same distribution as torch.randperm's,
        # 4 radix passes instead of 8 plus a duplicate-key pass)
        seed = torch.randint(-2 ** 63, 2 ** 63 - 1, (1,), device=self.device, dtype=torch.int64, generator=self.gen)
        return randperm(self.batch, seed)

    def _draw(self):
        self.left -= 1
        if self.side is None:
            return self._perm(), None
        main = torch.cuda.current_stream(self.device)
        self.side.wait_stream(main)  # the generator's state and the allocator: after what main queued so far
        with torch.cuda.stream(self.side):
            p = self._perm()
            ev = torch.cuda.Event()
            ev.record(self.side)
        return p, ev

    def next(self) -> torch.Tensor:
        p, ev = self.pending if self.pending is not None else self._draw()
        self.pending = None
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            p.record_stream(torch.cuda.current_stream(self.device))
        if self.side is not None and self.left > 0:
            self.pending = self._draw()  # the next epoch's, overlapping this epoch's minibatches
        return p


def ppo_update(agent, optimizer, flat, args, b_obs, b_logprobs, b_actions, b_advantages, b_returns,
               b_values, world=1, gen=None, graph=None):
    """Clipped PPO over update_epochs x num_minibatches (ppo…:306-365).  Returns last-minibatch
    stats.  `flat` holds the grads; with world > 1 it is all-reduced before clipping.  `graph` (a
    MinibatchGraph) replays the minibatch's forward and backward; None runs them eagerly."""
    device = b_obs.device
    batch = b_obs.shape[0]
    mb = batch // args.num_minibatches
    pad = padding_rows(mb, device)
    clipfracs = []
    epochs_run = 0
    # on the GPU with the Agent's networks: direct_minibatch (no autograd), captured or eager alike
    direct = device.type == "cuda" and MLP_ROW_PAD % 256 == 0 and direct_minibatch_ok(agent, args, flat)
    rows = {}  # eager direct flow: DirectRows per minibatch size
    global_stats = getattr(args, "global_adv_norm", True)
    perms = EpochPermutations(batch, device, gen, args.update_epochs, ahead=args.target_kl is None)
    for epoch in range(args.update_epochs):
        epochs_run += 1
        b_inds = perms.next()  # torch.randperm(batch) of ppo…:309, drawn from gen in epoch order
        for start in range(0, batch, mb):
            mb_inds = b_inds[start:start + mb]
            if direct and graph is not None and graph.direct and mb_inds.numel() == mb:
                st = graph.run_direct(mb_inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, world)
            elif direct:
                m = mb_inds.numel()
                m_pad = m + padding_rows(m, device)
                if m not in rows:
                    rows[m] = DirectRows(m, m_pad, b_obs[0].numel(), b_actions[0].numel(), device)
                r = rows[m]
                src = r.gather(mb_inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, args.norm_adv,
                               world, global_stats)
                _, st = direct_minibatch(agent, args, r.obs, r.act, r.logp, r.adv, *src, r.ret, r.val)
            else:
                # the networks' rows: the minibatch, then its first rows again up to the padding
                inds_pad = mb_inds
                if pad and mb_inds.numel() == mb:
                    inds_pad = torch.cat([mb_inds, mb_inds.repeat(-(-pad // mb))[:pad]])
                mb_adv = b_advantages[mb_inds]
                if args.norm_adv:
                    mb_adv = normalize_advantages(mb_adv, world, global_stats)
                if graph is not None:
                    st = graph.run(mb_inds, inds_pad, b_obs, b_actions, b_logprobs, mb_adv, b_returns, b_values)
                else:
                    loss, st = minibatch_losses(agent, args, b_obs[inds_pad], b_actions[inds_pad], b_logprobs[mb_inds],
                                                mb_adv, b_returns[mb_inds], b_values[mb_inds])
                    flat.zeroed_backward(loss)
            pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac = st
            clipfracs.append(clipfrac.clone())  # (a graph's outputs are rewritten by the next replay)
            flat.all_reduce_mean(world)  # the data-parallel exchange (RCCL on ROCm)
            flat.clip_norm_(args.max_grad_norm)
            optimizer.step()

            if args.adaptative_lr or args.target_kl is not None:
                if world > 1:
                    dist.all_reduce(approx_kl, op=dist.ReduceOp.SUM)
                    approx_kl /= world
            if args.adaptative_lr:
                optimizer.param_groups[0]["lr"] = adapted_lr(optimizer.param_groups[0]["lr"], float(approx_kl),
                                                             args.threshold_kl)
        if args.target_kl is not None and float(approx_kl) > args.target_kl:
            break
    return dict(v_loss=v_loss.detach().clone(), pg_loss=pg_loss.detach().clone(), entropy=entropy_loss.detach().clone(),
                old_approx_kl=old_approx_kl.clone(), approx_kl=approx_kl.clone(),
                clipfrac=torch.stack(clipfracs).mean(), epochs_run=epochs_run)


def setup_distributed():
    """One process per GPU (torch.distributed.run env). RCCL ("nccl") on GPUs, gloo on CPU.
    Rehearsal overrides (several ranks on one GPU): VSS_LOCAL_DEVICE pins the device index,
    VSS_DIST_BACKEND=gloo picks gloo (RCCL refuses two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device_index()
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("VSS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {"device_id": torch.device(f"cuda:{local}")} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def evaluate(args, unwrapped_env, checkpoint: str, writer, global_step: int) -> dict:
    """Post-training evaluation (ppo…:380-461) without W&B: goal-only rewards, the trained agent
    as the blue team against every baseline team available (play.py: zero, OU and the
    base_nets checkpoints present), `args.eval_matches` matches each; for SA also as 'sa-x3'
    (the single-agent policy controlling all three blue robots).  Scores go to the writer under
    the reference's Validation/* names and are returned."""
    from play import baseline_teams, get_team, play_matches
    unwrapped_env.w_goal, unwrapped_env.w_grad, unwrapped_env.w_move, unwrapped_env.w_energy = 1.0, 0.0, 0.0, 0.0
    device = unwrapped_env.device
    teams = baseline_teams(device=str(device))
    variants = [f"ppo-{args.env_id}"] + (["ppo-sa-x3"] if args.env_id == "sa" else [])
    out = {}
    for algo in variants:
        blue = get_team(algo, checkpoint, str(device))
        scores, lengths = [], []
        res = {}
        for team, seeds in teams.items():
            t_score = t_len = 0.0
            for seed, yellow in seeds.items():
                r, ln = play_matches(unwrapped_env, blue, yellow, args.eval_matches)
                t_score += r
                t_len += ln
                scores.append(r)
                lengths.append(ln)
            res[f"Validation/Score/{team}"] = t_score / len(seeds)
            res[f"Validation/Length/{team}"] = t_len / len(seeds)
        res["Validation/Score Mean"] = sum(scores) / len(scores)
        res["Validation/Length Mean"] = sum(lengths) / len(lengths)
        for k, v in res.items():
            writer.add_scalar(f"{algo}/{k}", v, global_step)
        print(f"evaluation {algo}: " + ", ".join(f"{k} {v:.3f}" for k, v in res.items()), flush=True)
        out[algo] = res
    return out


def warmup_kernels(args) -> float:
    """The first use of each torch kernel (and of the graph machinery) costs the runtime 10-200 ms of code-
    object loading (profiles/r05_first_updates_gaps.txt: hipLaunchKernel calls of up to 200 ms in the first
    update).  This runs train() once on a throwaway env and agent -- 16,384 envs (x 3 agent rows for DMA)
    x 8 steps, one update: the same code paths as the real loop (the rollout chain policy, the masked
    terminal values, GAE, the captured minibatch and its self-check, FlatAdam) at a small size -- and
    restores every RNG state afterwards, so the real run's results do not change.  Returns its seconds."""
    import copy
    t0 = time.perf_counter()
    rng = (random.getstate(), np.random.get_state(), torch.get_rng_state(),
           torch.cuda.get_rng_state_all() if torch.cuda.is_available() else None)
    w = copy.copy(args)
    w.num_envs = 3 * 16384 if args.env_id == "dma" else 16384
    w.num_steps, w.num_updates, w.total_timesteps = 8, 1, 0
    w.log, w.evaluate, w.capture_video, w.track, w.kernel_warmup = False, False, False, False, False
    w.batch_size = int(w.num_envs * w.num_steps)
    w.minibatch_size = int(w.batch_size // w.num_minibatches)
    train(w)
    random.setstate(rng[0])
    np.random.set_state(rng[1])
    torch.set_rng_state(rng[2])
    if rng[3] is not None:
        torch.cuda.set_rng_state_all(rng[3])
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def local_device_index() -> int:
    return int(os.environ.get("VSS_LOCAL_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def train(args, on_update=None):
    """The PPO loop (ppo…:231-379).  on_update(record, agent) -- optional, called after every update
    with that update's history record -- may return True to stop training early (tools/time_to_score.py
    evaluates the live policy there)."""
    disable_graph_packet_capture()  # effective only while nothing has initialised the GPU yet
    world, rank, local = setup_distributed()
    run_name = f"{args.exp_name}_ppo-{args.env_id}_{args.seed}"
    writer = make_writer(args, run_name, rank)
    writer.add_text("hyperparameters", "|param|value|\n|-|-|\n%s" % "\n".join(f"|{k}|{v}|" for k, v in vars(args).items()))

    seed = args.seed + rank
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(args.seed)  # same initial weights on every rank
    torch.backends.cudnn.deterministic = args.torch_deterministic
    device = torch.device(f"cuda:{local}" if torch.cuda.is_available() and args.cuda else "cpu")

    from envs.wrappers import RecordEpisodeStatisticsTorch, make_env
    unwrapped_env, envs = make_env(args)
    video = None
    if args.capture_video and rank == 0:  # ppo…:213-221 (GIF clips of field 0, envs/render.py)
        from envs.render import RecordVideo
        envs = video = RecordVideo(envs, f"{args.save_path}/{run_name}",
                                   step_trigger=lambda step: step % args.record_video_step_frequency == 0,
                                   video_length=100)
    envs = ExtractObsWrapper(envs)
    envs = RecordEpisodeStatisticsTorch(envs, device)
    envs.single_action_space = envs.action_space
    envs.single_observation_space = envs.observation_space
    assert isinstance(envs.single_action_space, Box), "only continuous action space is supported"

    agent = Agent(envs).to(device)
    flat = FlatGrads(agent, flat_params=device.type == "cuda")
    fused = None
    if args.fused_policy and device.type == "cuda" and args.amp == "none":
        from vss_amd.policy import FusedPolicy
        fused = FusedPolicy(agent, seed=seed * 7919 + 17)
    # torch's Adam (ppo…:166) -- on the GPU FlatAdam: the same update rule over the flat parameter and
    # gradient buffers, with the gradient clip, in one launch per minibatch (vss_adam_step_clipped)
    if device.type == "cuda":
        optimizer = FlatAdam(flat, lr=args.learning_rate, eps=1e-5)
    else:
        optimizer = optim.Adam(agent.parameters(), lr=args.learning_rate, eps=1e-5)
    gen = torch.Generator(device=device).manual_seed(seed)

    T, E = args.num_steps, args.num_envs
    obs_dim = envs.single_observation_space.shape
    act_dim = envs.single_action_space.shape
    obs = torch.zeros((T, E) + obs_dim, device=device)
    actions = torch.zeros((T, E) + act_dim, device=device)
    logprobs = torch.zeros((T, E), device=device)
    rewards = torch.zeros((T, E), device=device)
    next_dones = torch.zeros((T, E), device=device)
    next_timeouts = torch.zeros((T, E), device=device)
    values = torch.zeros((T, E), device=device)
    next_values = torch.zeros((T, E), device=device)
    term = TerminalValues(T, E, obs_dim, device) if fused is not None else None
    graph = make_minibatch_graph(agent, flat, args, T * E, obs_dim, act_dim, device)

    # outside the clock, as the reference's env and Agent construction before ppo…:244: the kernels' first
    # uses on a throwaway copy of the loop (warmup_kernels); args.kernel_warmup_s keeps the time it took
    args.kernel_warmup_s = warmup_kernels(args) if getattr(args, "kernel_warmup", False) and device.type == "cuda" \
        else 0.0
    global_step = 0
    start_time = time.time()
    next_obs = envs.reset()
    num_updates = args.num_updates if args.num_updates is not None else args.total_timesteps // (args.batch_size * world)
    history = []
    for update in range(1, num_updates + 1):
        if args.anneal_lr:
            optimizer.param_groups[0]["lr"] = annealed_lr(update, num_updates, args.learning_rate)
        t_roll = time.time()
        # per-env sums of finished episodes' returns and counts, reduced once after the rollout (two
        # elementwise launches per step instead of a product, two reductions and two adds)
        ep_ret = torch.zeros(E, device=device)
        ep_cnt = torch.zeros(E, device=device)
        # ppo…:273-279 logs the first finished env's episode stats at steps 0-2 (a host-sync loop);
        # here: [any done, goal, grad, move, energy, return, length] on the device, read once below
        ep_first = torch.zeros((3, 7), device=device)
        step0 = global_step
        if fused is not None:
            fused.refresh()  # weights changed in the last update
        for step in range(T):
            global_step += E * world
            obs[step] = next_obs
            if fused is not None:  # written straight into this step's storage rows
                action, _, _, _ = fused.get_action_and_value(next_obs, out=(actions[step], logprobs[step],
                                                                             values[step].view(E, 1)))
            else:
                with torch.no_grad(), autocast(args, device):
                    action, logprob, _, value = agent.get_action_and_value(next_obs)
                    values[step] = value.flatten()
                actions[step] = action.float()
                logprobs[step] = logprob.float()
            next_obs, rewards[step], next_done, info = envs.step(action)
            next_dones[step] = next_done
            next_timeouts[step] = info["time_outs"]
            if term is not None:  # critic(terminal obs) after the rollout (TerminalValues)
                term.record(step, info["terminal_observation"], next_done)
            else:
                with torch.no_grad(), autocast(args, device):
                    next_values[step] = agent.get_value(info["terminal_observation"]).reshape(1, -1)
            d = next_dones[step]  # next_done as float (the storage row just written)
            ep_ret.addcmul_(info["r"]["return"].reshape(E), d)
            ep_cnt.add_(d)
            if step <= 2:
                ep_first[step] = first_done_stats(d, info)
        if term is not None:
            next_values = term.next_values(fused, values, next_dones, next_obs)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t_roll = time.time() - t_roll
        if rank == 0 and args.log:
            for t, row in enumerate(ep_first.tolist()):
                if row[0] > 0:
                    gs = step0 + (t + 1) * E * world
                    for k, v in zip(EP_KEYS, row[1:6]):
                        writer.add_scalar(f"rws/episodic_{k}", v, gs)
                    writer.add_scalar("rws/episodic_length", row[6], gs)

        with torch.no_grad():
            advantages, returns = compute_gae(rewards, values, next_values, next_dones, next_timeouts,
                                              args.gamma, args.gae_lambda)
        t_upd = time.time()
        stats = ppo_update(agent, optimizer, flat, args, obs.reshape((-1,) + obs_dim), logprobs.reshape(-1),
                           actions.reshape((-1,) + act_dim), advantages.reshape(-1), returns.reshape(-1),
                           values.reshape(-1), world=world, gen=gen, graph=graph)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t_upd = time.time() - t_upd
        wall = time.time() - start_time
        sps = int(global_step / wall)
        rec = {"update": update, "global_step": global_step, "sps": sps, "wall_s": wall, "rollout_s": t_roll,
               "update_s": t_upd,
               "episodes": float(ep_cnt.sum()), "mean_return": float(ep_ret.sum() / ep_cnt.sum().clamp(min=1)),
               **{k: float(v) for k, v in stats.items()}}
        history.append(rec)
        for k, name in (("v_loss", "value_loss"), ("pg_loss", "policy_loss"), ("entropy", "entropy"),
                        ("old_approx_kl", "old_approx_kl"), ("approx_kl", "approx_kl"), ("clipfrac", "clipfrac")):
            writer.add_scalar(f"losses/{name}", rec[k], global_step)
        writer.add_scalar("losses/learning_rate", optimizer.param_groups[0]["lr"], global_step)
        writer.add_scalar("Charts/SPS", sps, global_step)
        if rank == 0 and args.log:
            print(f"update {update}/{num_updates} step {global_step} SPS {sps} rollout {t_roll:.2f}s "
                  f"update {t_upd:.2f}s return {rec['mean_return']:.3f} kl {rec['approx_kl']:.4f}", flush=True)
        if on_update is not None and on_update(rec, agent):
            break

    if rank == 0 and args.log:
        os.makedirs(f"{args.save_path}/{run_name}", exist_ok=True)
        torch.save(agent.state_dict(), f"{args.save_path}/{run_name}/{run_name}-agent.pt")
        wall = time.time() - start_time
        if args.evaluate:
            history.append({"validation": evaluate(args, unwrapped_env, f"{args.save_path}/{run_name}/{run_name}-agent.pt",
                                                   writer, global_step)})
        # the loss / SPS curves (what the reference sends to TensorBoard/W&B), one record per update
        with open(f"{args.save_path}/{run_name}/history.json", "w") as f:
            json.dump({"args": vars(args), "world": world, "wall_s": wall, "history": history}, f, indent=1)
    if video is not None:
        video.recorder.flush()  # a clip still open when training ends
    writer.close()
    return agent, history


if __name__ == "__main__":
    disable_graph_packet_capture()
    train(parse_args())
