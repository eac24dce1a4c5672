"""The Agent's MLPs in the PPO update (ppo_continuous_action_isaacgym.py:104-111,157-164 of the reference:
(Linear, Tanh) x L + Linear, forward and backward) on this repository's GEMM kernels.

    out = mlp_forward(seq, x)                         # _TanhMLP for the Agent's stacks, seq(x) otherwise
    action, logprob, entropy, value = get_action_and_value_update(agent, x, action)

UPDATE_GEMM "x6" (default, VSS_UPDATE_GEMM) runs the 256/512-wide layers in fp32 arithmetic on the bf16
matrix cores (csrc/vss_gemm_x6.hip; an exact 3-way bf16 split of every operand, error vs fp64 at or below
the fp32 GEMMs', tests/test_gemm_x6.py), "fp32" on the fp32-MFMA kernels (csrc/vss_update.hip).
(The round-4 A/B switches VSS_UPDATE_MLP=split, VSS_OUTPUT_FWD/BWD=0 and VSS_WEIGHT_PLANES=0, each strictly
slower, are retired from the product: tools/ab_switches_r04.patch re-adds them for A/B runs.)
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
from torch.distributions.normal import Normal

from .flat import grad_dst
from .update import (first_wgrad_ok, gemm_shape_ok, linear_tanh, linear_tanh_backward, linear_tanh_backward_mixed,
                     linear_tanh_mixed, linear_tanh_out, linear_tanh_out_mixed, linear_tanh_out_ok, output_backward,
                     output_backward_ok, sum_parts, weight_grad_mixed, weight_planes, x6_ok)

UPDATE_GEMM = os.environ.get("VSS_UPDATE_GEMM", "x6")

# The first layer's weight gradient dW = dY^T X reduces over all minibatch rows (2,097,152 at 65,536 envs)
# into a (256, 52) output; as one GEMM hipBLASLt runs it at ~1 TF.  Splitting the rows into SPLITK chunks
# (one batched GEMM + a sum) runs it at ~90 TF (tools/wgrad_bench.py); only the fp32 summation order differs.
SPLITK = 64
SPLITK_MIN_ROWS = 32768


def split_k_wgrad(gz, x, out=None):
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
    gradients as split GEMMs over the rows.  On the x6 GEMMs: whole 256-row tiles, the ragged rest of a
    minibatch on the fp32-MFMA kernels.  Inputs: x, W_0, b_0, ..., W_L, b_L."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        ctx.params = params  # the backward writes the FlatGrads-owned gradients in place (grad_dst)
        hs = [x]
        rows = x.shape[0]
        x6 = x.is_cuda and UPDATE_GEMM == "x6"
        # the x6 layers' weight planes, forward (W) and backward (W^T), in one launch for the whole MLP
        pf, ctx.planes_b = mlp_planes(ws, rows) if x6 else ({}, {})
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
        dst = [grad_dst(p) if gout.is_cuda else None for p in ctx.params]
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
        gz = backward_layers(hs, ws, ctx.planes_b, gz, gb, top, dst, grads, defer)
        if defer:
            sum_parts(defer)
        gx = gz.mm(ws[0]) if ctx.needs_input_grad[0] else None
        # the gradients already written into their parameters' .grad are not handed to autograd
        # (whose AccumulateGrad would add them to themselves)
        return (gx, *[None if d is not None else g for g, d in zip(grads, dst)])


def backward_layers(hs, ws, planes_b, gz, gb, top: int, dst, grads, defer):
    """Layers top, top - 1, ..., 0 of an MLP backward (_TanhMLP.backward, minibatch.direct_minibatch): gz =
    the pre-activation gradient of layer `top`, gb its bias gradient.  Each layer's weight gradient (x6
    kernels or the split-K GEMM) into dst / grads, then the backward into the tanh layer below with the tanh
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
            grads[2 * layer] = split_k_wgrad(gz, hs[layer], out=dst[2 * layer])
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


def mlp_planes(ws, rows: int):
    """The bf16 planes of the hidden layers' weights the x6 GEMMs take (vss_weight_planes_bf16x6, one
    launch): {layer: planes of W} for the forwards of layers 1 .. L-2 and {layer: planes of W^T} for
    their backwards (layer 0's input width is the observation's, below the x6 shapes; layer L-1 is the
    output layer).  Valid for this minibatch: the weights change only at the optimizer step."""
    return nets_planes([ws], rows)[0]


def nets_planes(nets, rows: int):
    """mlp_planes for several MLPs (nets = [their weight lists]) in one launch while the jobs fit it."""
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


def fused_mlp_ok(seq: nn.Sequential) -> bool:
    """Whether seq is the Agent's (Linear, Tanh) x L + Linear stack on shapes the fused kernels take."""
    mods = list(seq)
    if len(mods) < 3 or len(mods) % 2 == 0:
        return False
    lins, acts = mods[0::2], mods[1::2]
    if not all(type(m) is nn.Linear and m.bias is not None for m in lins) or \
            not all(isinstance(a, nn.Tanh) for a in acts):
        return False
    return all(gemm_shape_ok(m.in_features, m.out_features) for m in lins[:-1]) and \
        all(gemm_shape_ok((m.out_features + 3) // 4 * 4, m.in_features) for m in lins[1:])


def mlp_forward(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """The update's MLP: _TanhMLP for the Agent's (Linear, Tanh) x L + Linear stacks in fp32, the module
    itself (torch autograd) for anything else."""
    if x.dtype == torch.float32 and fused_mlp_ok(seq):
        params = [t for m in list(seq)[0::2] for t in (m.weight, m.bias)]
        return _TanhMLP.apply(x, *params)
    return seq(x)


def mlp_wb(seq: nn.Sequential):
    """([weights], [biases]) of an MLP's Linear layers, in order."""
    lins = list(seq)[0::2]
    return [m.weight for m in lins], [m.bias for m in lins]


def get_action_and_value_update(agent, x, action):
    """Agent.get_action_and_value (ppo…:157-164) on the same parameters, for the PPO update: the
    same function (forward within fp32 rounding: fused GEMM summation order and a few-ulp tanh),
    the MLPs through _TanhMLP."""
    mean = mlp_forward(agent.actor_mean, x)
    std = torch.exp(agent.actor_logstd.expand_as(mean))
    # no argument validation: its finiteness check is a host sync per minibatch, which a captured
    # minibatch (MinibatchGraph) cannot hold; the loss values are the same
    probs = Normal(mean, std, validate_args=False)
    return action, probs.log_prob(action).sum(1), probs.entropy().sum(1), mlp_forward(agent.critic, x)
