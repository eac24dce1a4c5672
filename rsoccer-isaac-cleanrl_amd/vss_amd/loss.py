"""The clipped PPO loss of one update minibatch (csrc/vss_loss.hip, include/vss.h vss_ppo_loss):

    loss, stats = ppo_loss(mean, logstd, value, action, logprob_old, adv, returns, values_old,
                           clip_coef, ent_coef, vf_coef, clip_vloss)

the reference's minibatch loss (ppo_continuous_action_isaacgym.py:318-349) from the networks' outputs:
`mean` (rows_pad, n_act) the actor's output, `logstd` (1, n_act) the Agent's actor_logstd, `value`
(rows_pad, 1) the critic's output, and the minibatch's stored rows (the first `rows` = len(logprob_old)
rows of the network outputs; rows beyond are padding the loss does not see).  `stats` = (pg_loss,
v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac), 0-dim tensors without gradient.  One autograd
node: the forward launch also writes d loss / d (mean, logstd, value), which the backward scales by the
incoming gradient.  On a ROCm device it runs the HIP kernels (and raises if the library is missing);
CPU tensors take the reference's torch expressions (`reference_loss`)."""
from __future__ import annotations

import torch
from torch.distributions.normal import Normal

from . import _native as N

N_ACT = (1, 2, 3, 4, 6, 8)


def reference_loss(mean, logstd, value, action, logprob_old, adv, returns, values_old, clip_coef, ent_coef, vf_coef,
                   clip_vloss):
    """The reference's expressions (ppo…:318-349; Agent.get_action_and_value ppo…:157-164), torch autograd."""
    n = logprob_old.shape[0]
    probs = Normal(mean, torch.exp(logstd.expand_as(mean)), validate_args=False)
    newlogprob = probs.log_prob(action).sum(1)[:n]
    entropy = probs.entropy().sum(1)[:n]
    newvalue = value[:n].view(-1)
    logratio = newlogprob - logprob_old
    ratio = logratio.exp()
    with torch.no_grad():
        old_approx_kl = (-logratio).mean()
        approx_kl = ((ratio - 1) - logratio).mean()
        clipfrac = ((ratio - 1.0).abs() > clip_coef).float().mean()
    pg_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip_coef, 1 + clip_coef)).mean()
    if clip_vloss:
        v_unclipped = (newvalue - returns) ** 2
        v_clipped = values_old + torch.clamp(newvalue - values_old, -clip_coef, clip_coef)
        v_loss = 0.5 * torch.max(v_unclipped, (v_clipped - returns) ** 2).mean()
    else:
        v_loss = 0.5 * ((newvalue - returns) ** 2).mean()
    entropy_loss = entropy.mean()
    loss = pg_loss - ent_coef * entropy_loss + v_loss * vf_coef
    return loss, (pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac)


def ppo_loss_ok(mean: torch.Tensor, value: torch.Tensor) -> bool:
    """Inputs the HIP loss takes: fp32 ROCm tensors, n_act in N_ACT, value one column."""
    return mean.is_cuda and mean.dtype == torch.float32 and value.dtype == torch.float32 and mean.dim() == 2 \
        and mean.shape[1] in N_ACT and value.numel() == mean.shape[0]


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mean, logstd, value, action, logprob_old, adv, returns, values_old, clip_coef, ent_coef, vf_coef,
                clip_vloss):
        rows, rows_pad, n_act = logprob_old.shape[0], mean.shape[0], mean.shape[1]
        lib = N.load()
        dev = mean.device
        f32 = dict(device=dev, dtype=torch.float32)
        mean, value, action = mean.contiguous(), value.contiguous(), action.contiguous()
        logstd_c = logstd.reshape(-1).contiguous()
        ins = [t.contiguous() for t in (logprob_old, adv, returns, values_old)]
        g_mean = torch.empty((rows_pad, n_act), **f32)
        g_value = torch.empty((rows_pad, 1), **f32)
        g_logstd = torch.empty((1, n_act), **f32)
        loss = torch.empty((), **f32)
        stats = torch.empty(6, **f32)
        part = torch.empty(lib.vss_ppo_loss_scratch_floats(rows_pad, n_act), **f32)
        c = float(clip_coef)  # ctypes rounds the clamp bounds to fp32 as torch.clamp does
        N.check(lib.vss_ppo_loss(N.stream_of(dev), rows, rows_pad, n_act, mean.data_ptr(), logstd_c.data_ptr(),
                                 value.data_ptr(), action.data_ptr(), *[t.data_ptr() for t in ins], c, 1 - c, 1 + c,
                                 float(ent_coef), float(vf_coef), int(bool(clip_vloss)), g_mean.data_ptr(),
                                 g_value.data_ptr(), g_logstd.data_ptr(), loss.data_ptr(), stats.data_ptr(),
                                 part.data_ptr()),
                "vss_ppo_loss")
        ctx.save_for_backward(g_mean, g_logstd, g_value)
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, g_loss, _g_stats):
        g_mean, g_logstd, g_value = ctx.saved_tensors
        return (g_mean * g_loss, g_logstd * g_loss, g_value * g_loss) + (None,) * 9


def ppo_loss(mean, logstd, value, action, logprob_old, adv, returns, values_old, clip_coef, ent_coef, vf_coef,
             clip_vloss):
    rows = logprob_old.shape[0]
    if mean.dim() != 2 or action.shape[1:] != mean.shape[1:] or action.shape[0] < rows or mean.shape[0] < rows \
            or value.shape[0] != mean.shape[0] or logstd.numel() != mean.shape[1] \
            or not (adv.shape == returns.shape == values_old.shape == logprob_old.shape):
        raise ValueError(f"ppo_loss: mean {tuple(mean.shape)}, value {tuple(value.shape)}, action {tuple(action.shape)}, "
                         f"logstd {tuple(logstd.shape)}, minibatch rows {tuple(logprob_old.shape)}")
    if not mean.is_cuda:
        return reference_loss(mean, logstd, value, action[:mean.shape[0]], logprob_old, adv, returns, values_old,
                              clip_coef, ent_coef, vf_coef, clip_vloss)
    if not ppo_loss_ok(mean, value) or rows == 0:
        raise ValueError(f"vss_ppo_loss: fp32 ROCm tensors with n_act in {N_ACT} and rows > 0 required, "
                         f"got {mean.dtype} {tuple(mean.shape)}")
    # the kernel reads every input as fp32 device memory: the action rows must cover the network rows
    # (padding included), and nothing may be a CPU, fp64 or other-device tensor
    if action.shape[0] < mean.shape[0]:
        raise ValueError(f"vss_ppo_loss: action has {action.shape[0]} rows, fewer than the {mean.shape[0]} network rows")
    for name, t in (("logstd", logstd), ("action", action), ("logprob_old", logprob_old), ("adv", adv),
                    ("returns", returns), ("values_old", values_old)):
        if t.dtype != torch.float32 or t.device != mean.device:
            raise ValueError(f"vss_ppo_loss: {name} must be fp32 on {mean.device}, got {t.dtype} on {t.device}")
    loss, stats = _PPOLoss.apply(mean, logstd, value.reshape(-1, 1), action[:mean.shape[0]], logprob_old, adv, returns,
                                 values_old, clip_coef, ent_coef, vf_coef, clip_vloss)
    return loss, tuple(stats[i] for i in range(6))


# ---- the update's minibatch without autograd (vss_amd/minibatch.py direct_minibatch) -------

def ppo_loss_direct(mean_parts, mean_bias, value_parts, value_bias, logstd, action, logprob_old, adv, adv_part,
                    adv_count, returns, values_old, clip_coef, ent_coef, vf_coef, clip_vloss, grad_logstd,
                    grad_mean_bias, grad_value_bias):
    """vss_ppo_loss_direct: the loss from the output layers' epilogue parts -- mean_parts (P, rows_pad,
    n_act) + mean_bias, value_parts (Q, rows_pad, 1) + value_bias -- and the RAW advantages, normalised in
    the kernel from adv_part ((parts, 2) fp64 (sum, sum of squares) over adv_count values; None: adv is
    used as given).  Writes d loss / d logstd and the output layers' bias gradients into grad_logstd,
    grad_mean_bias, grad_value_bias (the FlatGrads views); returns (grad_mean (rows_pad, n_act),
    grad_value (rows_pad, 1), loss, stats (6,))."""
    rows = logprob_old.shape[0]
    nm, rows_pad, n_act = mean_parts.shape
    nv = value_parts.shape[0]
    if n_act not in N_ACT or value_parts.shape[1] != rows_pad or value_parts.numel() != nv * rows_pad \
            or action.shape[0] < rows_pad or action.shape[1] != n_act or not 0 < rows <= rows_pad \
            or mean_bias.numel() != n_act or value_bias.numel() != 1 or logstd.numel() != n_act \
            or grad_logstd.numel() != n_act or grad_mean_bias.numel() != n_act or grad_value_bias.numel() != 1 \
            or not (adv.shape == returns.shape == values_old.shape == logprob_old.shape):
        raise ValueError(f"ppo_loss_direct: mean parts {tuple(mean_parts.shape)}, value parts {tuple(value_parts.shape)}, "
                         f"action {tuple(action.shape)}, rows {rows}")
    ts = (mean_parts, mean_bias, value_parts, value_bias, logstd, action, logprob_old, adv, returns, values_old,
          grad_logstd, grad_mean_bias, grad_value_bias)
    for t in ts:
        if t.dtype != torch.float32 or t.device != mean_parts.device or not t.is_contiguous():
            raise ValueError(f"ppo_loss_direct: contiguous fp32 tensors on {mean_parts.device}, got {t.dtype} on {t.device}")
    if adv_part is not None and (adv_part.dtype != torch.float64 or adv_part.device != mean_parts.device
                                 or adv_part.dim() != 2 or adv_part.shape[1] != 2 or not adv_part.is_contiguous()):
        raise ValueError("ppo_loss_direct: adv_part must be a contiguous (parts, 2) fp64 tensor on the same device")
    lib = N.load()
    dev = mean_parts.device
    f32 = dict(device=dev, dtype=torch.float32)
    g_mean = torch.empty((rows_pad, n_act), **f32)
    g_value = torch.empty((rows_pad, 1), **f32)
    loss = torch.empty((), **f32)
    stats = torch.empty(6, **f32)
    part = torch.empty(lib.vss_ppo_loss_direct_scratch_floats(rows_pad, n_act), **f32)
    c = float(clip_coef)
    N.check(lib.vss_ppo_loss_direct(
        N.stream_of(dev), rows, rows_pad, n_act, mean_parts.data_ptr(), nm, mean_bias.data_ptr(), value_parts.data_ptr(),
        nv, value_bias.data_ptr(), logstd.data_ptr(), action.data_ptr(), logprob_old.data_ptr(), adv.data_ptr(),
        adv_part.data_ptr() if adv_part is not None else None, adv_part.shape[0] if adv_part is not None else 0,
        float(adv_count), returns.data_ptr(), values_old.data_ptr(), c, 1 - c, 1 + c, float(ent_coef), float(vf_coef),
        int(bool(clip_vloss)), g_mean.data_ptr(), g_value.data_ptr(), grad_logstd.data_ptr(), grad_mean_bias.data_ptr(),
        grad_value_bias.data_ptr(), loss.data_ptr(), stats.data_ptr(), part.data_ptr()), "vss_ppo_loss_direct")
    return g_mean, g_value, loss, stats


def ppo_loss_fused_finish(actor_stats, critic_stats, rows: int, logstd, ent_coef, vf_coef, grad_logstd,
                          grad_mean_bias, grad_value_bias):
    """vss_ppo_loss_fused_finish: the per-block loss sums of the actor's and the critic's fused loss
    launches (update.linear_tanh_loss_x6) -> (loss, stats (6,)); writes d loss / d logstd and the output
    layers' bias gradients into grad_logstd, grad_mean_bias, grad_value_bias as ppo_loss_direct."""
    n_act = logstd.numel()
    for t in (actor_stats, critic_stats, logstd, grad_logstd, grad_mean_bias, grad_value_bias):
        if t.dtype != torch.float32 or t.device != actor_stats.device or not t.is_contiguous():
            raise ValueError("ppo_loss_fused_finish: contiguous fp32 tensors on one device")
    if actor_stats.device.type != "cuda":
        raise ValueError("ppo_loss_fused_finish: ROCm tensors only (no CPU path)")
    if n_act not in (1, 2) or actor_stats.dim() != 2 or actor_stats.shape[1] != 32 or critic_stats.dim() != 2 \
            or critic_stats.shape[1] != 32 or grad_logstd.numel() != n_act or grad_mean_bias.numel() != n_act \
            or grad_value_bias.numel() != 1 or rows <= 0:
        raise ValueError(f"ppo_loss_fused_finish: stats {tuple(actor_stats.shape)} / {tuple(critic_stats.shape)}, "
                         f"{n_act} actions")
    f32 = dict(device=actor_stats.device, dtype=torch.float32)
    loss, stats = torch.empty((), **f32), torch.empty(6, **f32)
    N.check(N.load().vss_ppo_loss_fused_finish(
        N.stream_of(actor_stats.device), rows, n_act, actor_stats.shape[0], actor_stats.data_ptr(), critic_stats.shape[0],
        critic_stats.data_ptr(), logstd.data_ptr(), float(ent_coef), float(vf_coef), grad_logstd.data_ptr(),
        grad_mean_bias.data_ptr(), grad_value_bias.data_ptr(), loss.data_ptr(), stats.data_ptr()),
        "vss_ppo_loss_fused_finish")
    return loss, stats


def randperm(n: int, seed: torch.Tensor, key_bits: int = 32) -> torch.Tensor:
    """A uniformly random permutation of [0, n) (int64, on seed's device) determined by seed, one int64 on
    the ROCm device drawn from the update's generator (vss_randperm: 32 random bits per index, a 4-pass
    radix sort, every run of tied bits shuffled) -- torch.randperm(n) of ppo…:309 in half its sort passes.
    key_bits < 32 draws fewer random bits per index, forcing ties (tests of the tie pass)."""
    if seed.dtype != torch.int64 or seed.numel() != 1 or seed.device.type != "cuda" or not 0 < n < 2 ** 31 \
            or not 1 <= key_bits <= 32:
        raise ValueError(f"randperm: n in (0, 2^31), key_bits in [1, 32] and a one-element int64 ROCm seed, got {n}, "
                         f"{key_bits}, {seed.dtype} {tuple(seed.shape)} on {seed.device}")
    lib = N.load()
    nb = int(lib.vss_randperm_scratch_bytes(n))
    scratch = torch.empty(nb, dtype=torch.uint8, device=seed.device)
    out = torch.empty(n, dtype=torch.int64, device=seed.device)
    N.check(lib.vss_randperm_bits(N.stream_of(seed.device), n, int(key_bits), seed.data_ptr(), out.data_ptr(),
                                  scratch.data_ptr(), nb), "vss_randperm_bits")
    return out


def minibatch_gather_parts(mb: int) -> int:
    """Rows of the (sum, sum of squares) parts minibatch_gather writes for mb minibatch rows."""
    return int(N.load().vss_minibatch_gather_parts(mb))


def minibatch_gather(inds, b_obs, b_act, b_logp, b_adv, b_ret, b_val, obs, act, logp, adv, ret, val, adv_part):
    """vss_minibatch_gather: the minibatch rows inds (int64, mb) of the batch tensors into obs / act
    (rows_pad >= mb rows: the padding rows repeat the minibatch's) and logp / adv / ret / val (mb), with
    the advantages' fp64 (sum, sum of squares) parts in adv_part ((minibatch_gather_parts(mb), 2)), in one
    launch (ppo…:310-317 b_obs[mb_inds] ... and the sums of ppo…:325-326's normalisation)."""
    mb, rows_pad, batch = inds.numel(), obs.shape[0], b_obs.shape[0]
    bo, ba = b_obs.reshape(batch, -1), b_act.reshape(batch, -1)
    ow, aw = bo.shape[1], ba.shape[1]
    f32 = (b_obs, b_act, b_logp, b_adv, b_ret, b_val, obs, act, logp, adv, ret, val)
    if inds.dtype != torch.int64 or not inds.is_contiguous() or not inds.is_cuda or rows_pad < mb or mb == 0 \
            or obs.reshape(rows_pad, -1).shape[1] != ow or act.shape[0] != rows_pad or act.reshape(rows_pad, -1).shape[1] != aw \
            or any(t.numel() != mb for t in (logp, adv, ret, val)) or any(t.shape[0] != batch for t in f32[:6]) \
            or adv_part.dtype != torch.float64 or adv_part.numel() != 2 * minibatch_gather_parts(mb) \
            or any(t.dtype != torch.float32 or not t.is_contiguous() or t.device != inds.device for t in f32):
        raise ValueError(f"minibatch_gather: {mb} indices into a batch of {batch} x {ow} / {aw}, outputs of "
                         f"{rows_pad} rows")
    N.check(N.load().vss_minibatch_gather(N.stream_of(inds.device), mb, rows_pad, batch, inds.data_ptr(), ow, aw,
                                          *[t.data_ptr() for t in f32], adv_part.data_ptr()), "vss_minibatch_gather")


def adv_part_sum(adv_part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out (1, 2) fp64 = adv_part's rows summed in order (the data-parallel all-reduce's operand)."""
    if adv_part.dtype != torch.float64 or out.dtype != torch.float64 or out.numel() != 2 or adv_part.dim() != 2:
        raise ValueError("adv_part_sum: fp64 (parts, 2) -> (1, 2)")
    N.check(N.load().vss_adv_part_sum(N.stream_of(out.device), adv_part.shape[0], adv_part.data_ptr(), out.data_ptr()),
            "vss_adv_part_sum")
    return out
