"""One PPO update minibatch on the GPU (ppo_continuous_action_isaacgym.py:306-354 of the reference: the
epoch's permutation, the minibatch rows, the networks, the clipped losses, loss.backward()).

    perms = EpochPermutations(batch, device, gen, epochs)       # torch.randperm(batch) per epoch (ppo…:309)
    graph = make_minibatch_graph(agent, flat, args, batch, ...)  # None: eager
    st = graph.run_direct(inds, b_obs, ..., world)              # gather + forward + loss + backward, replayed

On a ROCm device each minibatch is ONE fixed sequence of this repository's launches (direct_minibatch), not
an autograd graph: one gather launch for the rows and the advantages' fp64 sums (vss_minibatch_gather), the
hidden layers on the x6 GEMMs, each network's loss terms and output-layer backward inside its last hidden
layer's launch (vss_linear_tanh_loss_bf16x6 + vss_ppo_loss_fused_finish; VSS_FUSED_LOSS=0 keeps the separate
vss_ppo_loss_direct / vss_output_backward_direct launches), every gradient written into its FlatGrads view,
captured once as a HIP graph (MinibatchGraph) and replayed.  The autograd path (minibatch_losses +
FlatGrads.zeroed_backward) runs on the CPU, under --amp bf16 and for networks outside those shapes.
"""
from __future__ import annotations

import os
import warnings

import numpy as np
import torch
import torch.distributed as dist

from . import mlp as M
from .loss import (N_ACT, adv_part_sum, minibatch_gather, minibatch_gather_parts, ppo_loss, ppo_loss_direct,
                   ppo_loss_fused_finish, randperm)
from .update import (linear_tanh_loss_x6, linear_tanh_loss_x6_ok, linear_tanh_mixed, linear_tanh_out_x6,
                     output_backward_direct, output_backward_direct_ok, sum_parts, x6_ok)

# direct_minibatch's loss folded into the last hidden layer's x6 launch (vss_linear_tanh_loss_bf16x6) where
# the output layers allow it; "0" keeps the separate output-layer / loss / output-backward launches
FUSED_LOSS = os.environ.get("VSS_FUSED_LOSS", "1") != "0"
# the epochs' permutations: torch.randperm from the update's generator (the reference's ppo…:309, default);
# VSS_RANDPERM=hip draws them with vss_randperm from one seed per epoch (measured within noise of torch's:
# 2.2615 vs 2.2645 s per update, profiles/r05_randperm_ab.log)
RANDPERM_HIP = os.environ.get("VSS_RANDPERM", "torch") == "hip"
# the update's minibatch rows are padded to a multiple of this on the GPU, so that every hidden-layer GEMM
# runs on whole x6 tiles: at 4,095 envs a 131,040-row minibatch otherwise leaves 224-row tails that
# hipBLASLt runs on one or two workgroups (43-110 us each, ~21 ms per update)
MLP_ROW_PAD = 256
# MinibatchGraph re-runs replays 12, 48, 192, ... (GRAPH_CHECK_REPLAY x GRAPH_CHECK_FACTOR^m) eagerly and
# compares each with its replay bit for bit: round 3's packet-capture failure began at the 9th replay
# (profiles/r03w_graph_probe2.log), and a later onset is caught at the next check; the checks cost one eager
# minibatch each, O(log replays) per run
GRAPH_CHECK_REPLAY = 12
GRAPH_CHECK_FACTOR = 4

# ---- ROCm's graph packet capture -------------------------------------------------------------------------
# In round 3 a captured 2,097,152-row minibatch replayed wrongly from its 9th launch on with it on
# (profiles/r03w_graph_probe2.log); in round 4 neither the same code (commit ea0c048) nor this tree
# reproduces that on any MLP / loss path, torch-only included (tools/graph_replay_probe.py,
# profiles/r04_graph_replay_probes.log), so the defect is not this repository's kernels and is not
# reproducible on demand.  The entry points start the runtime with it off (disable_graph_packet_capture);
# importing a module changes no environment variable, and every captured minibatch is guarded by
# MinibatchGraph's self-check against eager.  The runtime reads the switch once, when it initialises: what
# counts is the value at that moment, which this module records while the GPU is still uninitialised.
PACKET_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
_SEEN_BEFORE_INIT = {"value": None, "seen": False}


def _note_packet_capture():
    """Record the switch's value while nothing has initialised the GPU (the latest such observation)."""
    if not torch.cuda.is_initialized():
        _SEEN_BEFORE_INIT["value"] = os.environ.get(PACKET_CAPTURE)
        _SEEN_BEFORE_INIT["seen"] = True


def _startup_environment_value():
    """The switch in the environment the process was started with (/proc/self/environ), or None."""
    try:
        with open("/proc/self/environ", "rb") as f:
            for item in f.read().split(b"\0"):
                if item.startswith(PACKET_CAPTURE.encode() + b"="):
                    return item.split(b"=", 1)[1].decode()
    except OSError:
        pass
    return None


def disable_graph_packet_capture() -> bool:
    """Entry points call this before anything initialises the GPU (the runtime reads the switch when it
    starts): sets DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 unless the environment already chose.  Returns
    whether the switch is now off."""
    if PACKET_CAPTURE not in os.environ and not torch.cuda.is_initialized():
        os.environ[PACKET_CAPTURE] = "0"
    _note_packet_capture()
    return os.environ.get(PACKET_CAPTURE) == "0"


def packet_capture_off_at_init() -> bool:
    """Whether the HIP runtime started with graph packet capture off: the switch was "0" when this module
    last saw it before the GPU initialised (or, if it never did, in the process's startup environment),
    and it is still "0" now.  False when unknown."""
    if os.environ.get(PACKET_CAPTURE) != "0":
        return False
    if _SEEN_BEFORE_INIT["seen"]:
        return _SEEN_BEFORE_INIT["value"] == "0"
    return _startup_environment_value() == "0"


_note_packet_capture()  # at import: if the GPU is not initialised yet, the value it will start with so far


# ---- the minibatch, autograd form ------------------------------------------------------------------------

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


def minibatch_losses(agent, args, obs, actions, logprobs, adv, returns, values):
    """The clipped PPO losses of ppo…:318-349 on one minibatch (adv already normalised when
    --norm-adv): (loss, (pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac)).
    obs / actions may carry padding rows beyond the minibatch's len(logprobs) (copies of its first
    rows): the networks run over them, the losses do not see them, so their gradient is zero."""
    if getattr(args, "amp", "none") == "none":
        # the networks (_TanhMLP on the GPU) ...
        mean = M.mlp_forward(agent.actor_mean, obs)
        value = M.mlp_forward(agent.critic, obs)
    else:  # --amp bf16: the networks under autocast, the loss in fp32
        with autocast(args, obs.device):
            mean, value = agent.actor_mean(obs), agent.critic(obs)
        mean, value = mean.float(), value.float()
    # ... then the loss and its gradients into the networks' outputs as one autograd node (vss_ppo_loss:
    # two launches on the GPU instead of ~100; the reference's expressions on the CPU)
    return ppo_loss(mean, agent.actor_logstd, value, actions, logprobs, adv, returns, values, args.clip_coef,
                    args.ent_coef, args.vf_coef, args.clip_vloss)


# ---- the minibatch without autograd (round 5) ------------------------------------------------------------
# The output layers' epilogue parts go straight into the loss (no sum / bias-add launches, the advantage
# normalisation and the output biases' gradients inside it), the loss's row gradients straight into the
# output layers' backward (no padded copies, no autograd scaling by the loss's incoming gradient of 1), and
# every gradient is written into its FlatGrads view (no zeroing, no AccumulateGrad).  The kernels are those
# of the autograd path (_TanhMLP); the results differ from it by summation order only
# (tests/test_direct_minibatch.py), and from fp64 autograd of the reference's expressions by at most the
# fp32 error of torch's own autograd (tests/test_update_parity.py).

def direct_minibatch_ok(agent, args, flat) -> bool:
    """Whether the update's minibatches run as direct_minibatch: x6 GEMMs, fp32 (no --amp), both MLPs the
    Agent's (Linear, Tanh) x L + Linear stacks with a 256-wide last hidden layer on the x6 shapes (its
    output layer's parts feed the loss: 1, 2 or 6 outputs, the actor's n_act in the loss's set, the critic
    one value), and every parameter's .grad a FlatGrads view on the GPU."""
    if flat is None or M.UPDATE_GEMM != "x6" or getattr(args, "amp", "none") != "none":
        return False
    for seq, outs in ((agent.actor_mean, N_ACT), (agent.critic, (1,))):
        if not M.fused_mlp_ok(seq):
            return False
        ws, _ = M.mlp_wb(seq)
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


def fused_loss_ok(agent, rows_pad: int) -> bool:
    """Whether direct_minibatch folds the loss into the last hidden layers' launches: the actor's 1 or 2
    outputs, the critic's value (direct_minibatch_ok's networks otherwise)."""
    for seq in (agent.actor_mean, agent.critic):
        ws, _ = M.mlp_wb(seq)
        (n, k), k_out = ws[-2].shape, ws[-1].shape[0]
        if not linear_tanh_loss_x6_ok(rows_pad, k, n, k_out):
            return False
    return M.mlp_wb(agent.critic)[0][-1].shape[0] == 1


def direct_minibatch(agent, args, obs, act, logp, adv, adv_part, adv_count, ret, val):
    """One update minibatch (ppo…:331-352: the networks, the clipped losses, loss.backward() into the
    zeroed gradients) as a fixed launch sequence writing every gradient into its FlatGrads view.  obs / act
    (rows_pad rows, the padding repeating the minibatch), logp / adv / ret / val (rows); adv RAW, normalised
    inside the loss from adv_part / adv_count (vss_ppo_loss_direct; None: as given).  Returns (loss,
    (pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac))."""
    (pfa, pba), (pfc, pbc) = M.nets_planes([M.mlp_wb(agent.actor_mean)[0], M.mlp_wb(agent.critic)[0]], obs.shape[0])
    planes = {id(agent.actor_mean): (pfa, pba), id(agent.critic): (pfc, pbc)}

    def forward(seq):
        ws, bs = M.mlp_wb(seq)
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
        M.backward_layers(hs, ws, pb, gz, gb, n - 2, d, [None] * (2 * n), defer)

    def fused(seq, is_actor, defer):
        # the hidden layers below the last, then the last hidden layer + output layer + this network's loss
        # terms + the output layer's backward in one launch
        ws, bs = M.mlp_wb(seq)
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
    if FUSED_LOSS and fused_loss_ok(agent, obs.shape[0]):
        with torch.no_grad():
            defer = []
            a_net, a_st = fused(agent.actor_mean, True, defer)
            c_net, c_st = fused(agent.critic, False, defer)
            loss, stats = ppo_loss_fused_finish(a_st, c_st, logp.shape[0], agent.actor_logstd, args.ent_coef,
                                                args.vf_coef, agent.actor_logstd.grad, a_net[6][-1], c_net[6][-1])
            for hs, ws, pb, gz, gb, n, d in (a_net, c_net):
                M.backward_layers(hs, ws, pb, gz, gb, n - 2, d, [None] * (2 * n), defer)
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


def padding_rows(mb: int, device) -> int:
    """Rows the update adds to a minibatch of mb rows (MLP_ROW_PAD on a ROCm GPU, none on the CPU)."""
    return (-mb) % MLP_ROW_PAD if torch.device(device).type == "cuda" else 0


def graph_check_due(replays: int) -> bool:
    """Whether replay number `replays` (1-based) of a MinibatchGraph is re-run eagerly and compared."""
    r = GRAPH_CHECK_REPLAY
    while r < replays:
        r *= GRAPH_CHECK_FACTOR
    return r == replays


class MinibatchGraph:
    """One minibatch's forward, losses and backward (into FlatGrads) captured once as a HIP graph and
    replayed for every minibatch: the ~30 launches of a direct minibatch (~300 for the autograd form)
    become one graph launch.  At the reference's 4,095 envs the update is launch-bound -- 131,040-row
    minibatches, the GPU idle ~23 % of it eagerly (profiles/r03w_trace_summary.txt).  The gathers into the
    static inputs, the advantage statistics' all-reduce when world > 1, the gradient all-reduce, clipping
    and the optimizer step run eagerly around the replay, so the learning-rate schedules apply unchanged.
    The kernels and their order are the eager path's, so the results are the same bits (tests/test_ppo.py).

    Device memory: the eager minibatches (the first, and the self-checks) and the captured one allocate
    their intermediates from ONE private memory pool (a torch.cuda.MemPool shared by the capture and by the
    eager runs), so a minibatch's activations and gradients are held once, not once per allocator pool --
    ~100 GB for a minibatch of DMA config 4 (see DESIGN.md §7 on the first update's allocation cost)."""

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
        self.pool = torch.cuda.MemPool() if SHARED_POOL and torch.device(device).type == "cuda" else None
        # the eager minibatches and the capture on ONE stream: the caching allocator hands a freed block only to
        # allocations on the stream it was freed on, so with the eager runs on the current stream and the capture
        # on torch.cuda.graph's own one the pool held two copies of the minibatch (216 of 232 GiB reserved against
        # a 109 GiB peak of live tensors for DMA config 4, profiles/r06zd_memory_dma.log)
        self.stream = torch.cuda.Stream(device=device) if self.pool is not None else None

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

    def _eager(self):
        """The minibatch eagerly, its intermediates from the graph's pool on the capture's stream (freed at
        return, reused by the capture, the replays and the next eager run in stream order)."""
        if self.pool is None:
            return self._body()
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream), torch.cuda.use_mem_pool(self.pool):
            out = self._body()
        cur.wait_stream(self.stream)
        return out

    def _capture(self):
        torch.cuda.synchronize()
        if self.pool is None:
            # the first minibatch ran eagerly from the default pool (library handles, workspaces, lazy
            # initialisation); release its cached blocks only when the device could not hold a second copy
            # of them beside the graph's private pool
            free, _ = torch.cuda.mem_get_info()
            if free < 1.25 * (torch.cuda.memory_reserved() - torch.cuda.memory_allocated()):
                torch.cuda.empty_cache()
        g = torch.cuda.CUDAGraph()
        # thread_local: with several ranks, RCCL's and the process group's own threads keep querying
        # their streams and events while this thread captures (no collective is captured)
        with torch.cuda.graph(g, pool=self.pool.id if self.pool is not None else None, stream=self.stream,
                              capture_error_mode="thread_local"):
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

    def prepare(self, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values, world: int = 1):
        """Set-up before the train clock (ppo…:244), like the reference's storage allocation before it: the
        eager first minibatch and the capture, on the first rows of the (not yet filled) rollout storage, so
        the minibatch's device memory -- ~100 GB for DMA config 4 -- is allocated, and the graph captured,
        outside the timed loop.  The gradients it writes are zeroed; no parameter, optimizer state or RNG
        changes.  Every real minibatch then replays (the same kernels in the same order: the same bits).
        Direct flow only; with several ranks every rank calls it (the advantage statistics' all-reduce)."""
        if not self.direct or self.graph is not None or self.failed:
            return
        mb = self.logp.numel()
        inds = torch.arange(mb, device=self.logp.device)
        self.adv_src = self.rows.gather(inds, b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values,
                                        self.args.norm_adv, world, getattr(self.args, "global_adv_norm", True))
        self.warm = True
        self._eager()
        self._capture()
        self.flat.zero()
        torch.cuda.synchronize()

    def _step(self):
        if self.failed:
            return self._eager()
        if self.graph is None:
            if not self.warm:  # the first minibatch: eager, real work
                self.warm = True
                return self._eager()
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
        want = list(self._eager())
        same = all(torch.equal(a, b) for a, b in zip(got, want + [self.flat.flat]))
        if same:
            return self.out
        warnings.warn(f"MinibatchGraph: replay {self.replays} differs from the eager minibatch; the update runs "
                      f"eagerly from here on ({PACKET_CAPTURE}={os.environ.get(PACKET_CAPTURE, '<unset>')})",
                      RuntimeWarning)
        self.failed, self.graph = True, None
        return tuple(want)


# eager minibatches in the captured graph's memory pool (MinibatchGraph); VSS_SHARED_POOL=0: the default pool
SHARED_POOL = os.environ.get("VSS_SHARED_POOL", "1") != "0"
_WARNED_PACKET_CAPTURE = [False]


def make_minibatch_graph(agent, flat, args, batch, obs_dim, act_dim, device):
    """MinibatchGraph when --update-graph applies (ROCm GPU, fp32, equal minibatches, and the runtime
    started with graph packet capture off), else None: the update then runs eagerly."""
    mb = batch // args.num_minibatches
    if not getattr(args, "update_graph", False) or torch.device(device).type != "cuda" or \
            getattr(args, "amp", "none") != "none" or batch % mb:
        return None
    if not packet_capture_off_at_init():
        # a runtime that started with packet capture on (or a caller that initialised the GPU before
        # disable_graph_packet_capture()): no capture -- round 3's corrupted replays ran in that mode
        # (profiles/r03w_graph_probe2.log)
        if not _WARNED_PACKET_CAPTURE[0]:
            warnings.warn(f"{PACKET_CAPTURE}={os.environ.get(PACKET_CAPTURE, '<unset>')}: the runtime did not "
                          "provably start with graph packet capture off, so the update minibatches run eagerly (call "
                          "disable_graph_packet_capture() before anything initialises the GPU)", RuntimeWarning)
            _WARNED_PACKET_CAPTURE[0] = True
        return None
    return MinibatchGraph(agent, flat, args, mb, obs_dim, act_dim, device)


_SIDE_STREAMS = {}


class EpochPermutations:
    """The update's per-epoch minibatch permutations (ppo…:309: torch.randperm(batch) from `gen`, in epoch
    order; with VSS_RANDPERM=hip vss_randperm from one seed per epoch drawn from `gen`).  On a ROCm device with
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
        # vss_randperm from one seed drawn from gen (a uniform permutation: 32 random bits per index, tied
        # keys shuffled, csrc/vss_loss.hip)
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


def warmup_kernels(args, train) -> float:
    """The first use of each torch kernel (and of the graph machinery) costs the runtime 10-200 ms of code-
    object loading (profiles/r05_first_updates_gaps.txt: hipLaunchKernel calls of up to 200 ms in the first
    update).  This runs train(args) once on a throwaway env and agent -- 16,384 envs (x 3 agent rows for DMA)
    x 8 steps, one update: the same code paths as the real loop (the rollout chain policy, the masked
    terminal values, GAE, the captured minibatch and its self-check, FlatAdam) at a small size -- and
    restores every RNG state afterwards, so the real run's results do not change.  Returns its seconds."""
    import copy
    import random
    import time
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


__all__ = ["FUSED_LOSS", "RANDPERM_HIP", "MLP_ROW_PAD", "GRAPH_CHECK_REPLAY", "GRAPH_CHECK_FACTOR", "PACKET_CAPTURE",
           "disable_graph_packet_capture", "packet_capture_off_at_init", "autocast", "normalize_advantages",
           "minibatch_losses", "direct_minibatch_ok", "fused_loss_ok", "direct_minibatch", "DirectRows",
           "padding_rows", "graph_check_due", "MinibatchGraph", "make_minibatch_graph", "EpochPermutations",
           "warmup_kernels"]
