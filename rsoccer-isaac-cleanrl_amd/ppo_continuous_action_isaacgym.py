"""Drop-in PPO train loop (cleanrl ppo_continuous_action_isaacgym, as used by the reference's
ppo_continuous_action_isaacgym.py) on the MI355X VSS env.

Same command line (`--env-id sa|cma|dma --num-envs ... --num-steps ...`, ppo…:48-118), same
`Agent` (module order, orthogonal init, state-dict keys: ppo…:121-164), same rollout / GAE /
clipped-PPO update semantics (ppo…:231-365).  This file keeps the reference's shape -- argparse, Agent,
the loop -- and the machinery under it lives in vss_amd/:

* the env is the fused HIP step (envs/wrappers.py), one launch per control step; the rollout policy is
  vss_amd.policy.FusedPolicy, its terminal values vss_amd.policy.TerminalValues;
* each update minibatch (ppo…:310-352) is vss_amd.minibatch: one fixed launch sequence without autograd on
  the GPU (direct_minibatch), captured as a HIP graph (MinibatchGraph), the permutations from
  EpochPermutations (torch.randperm from the update's generator, as ppo…:309);
* parameters and gradients are flat buffers (vss_amd.flat.FlatGrads), stepped by FlatAdam (clip + Adam in
  one launch);
* data parallel over ranks (one process per GPU, `torch.distributed` = RCCL): each rank owns
  `--num-envs` environments (weak scaling; BASELINE config 5 = 8 x 65,536) and its own rollout
  storage; the only exchange is ONE all-reduce of the flat fp32 gradient buffer per minibatch,
  between backward() and clip_grad_norm_ (ppo…:352-353), plus the advantage statistics' 16 B when
  --norm-adv normalises over all ranks' rows; approx_kl is averaged over ranks when it drives a decision;
* no per-element host-synchronising logging loop (ppo…:273-279): episode statistics are
  reduced on the device and read once per update;
* logging is optional (TensorBoard if installed, else a CSV of the same scalars; no W&B).
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
import torch.nn as nn
import torch.optim as optim
from torch.distributions.normal import Normal

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from envs._gym import Box, ObservationWrapper  # noqa: E402
from vss_amd import minibatch as MB  # noqa: E402
from vss_amd.flat import FlatAdam, FlatGrads  # noqa: E402,F401
from vss_amd.minibatch import (DirectRows, EpochPermutations, autocast, direct_minibatch,  # noqa: E402,F401
                               direct_minibatch_ok, disable_graph_packet_capture, make_minibatch_graph,
                               minibatch_losses, normalize_advantages, padding_rows, warmup_kernels)
from vss_amd.mlp import get_action_and_value_update  # noqa: E402,F401
from vss_amd.writers import make_writer  # noqa: E402

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
                        "(vss_amd.minibatch.MinibatchGraph; on a ROCm GPU with --amp none), eager otherwise")
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


class ExtractObsWrapper(ObservationWrapper):
    def observation(self, obs):
        return obs["obs"]


EP_KEYS = ("goal", "grad", "move", "energy", "return")  # info['r'] keys (envs/wrappers.py:74-80)


def first_done_stats(done: torch.Tensor, info: dict) -> torch.Tensor:
    """[any done, goal, grad, move, energy, return, length] of the FIRST env with done set — what
    ppo…:273-279 logs by looping over the envs on the host — as one device tensor, no sync."""
    d = done.float()
    idx = torch.argmax(d)  # index of the first maximum
    return torch.stack([d.max()] + [info["r"][k][idx].float() for k in EP_KEYS] + [info["l"][idx].float()])


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
    direct = device.type == "cuda" and MB.MLP_ROW_PAD % 256 == 0 and direct_minibatch_ok(agent, args, flat)
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
    if torch.cuda.is_available():
        torch.cuda.set_device(local)  # before the process group: nothing touches another rank's GPU
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("VSS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {"device_id": torch.device(f"cuda:{local}")} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return world, rank, local


def local_device_index() -> int:
    return int(os.environ.get("VSS_LOCAL_DEVICE", os.environ.get("LOCAL_RANK", "0")))


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
        from vss_amd.policy import FusedPolicy, TerminalValues
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
    args.kernel_warmup_s = warmup_kernels(args, train) if getattr(args, "kernel_warmup", False) and device.type == "cuda" \
        else 0.0
    # and the update minibatch's device memory and graph capture (MinibatchGraph.prepare), on the empty storage
    t_prep = time.perf_counter()
    if graph is not None:
        graph.prepare(obs.reshape((-1,) + obs_dim), actions.reshape((-1,) + act_dim), logprobs.reshape(-1),
                      values.reshape(-1), values.reshape(-1), values.reshape(-1), world)
    args.graph_prepare_s = time.perf_counter() - t_prep
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
