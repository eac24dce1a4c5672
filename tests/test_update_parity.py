"""The product's default update path pinned directly against the reference's expressions (round-5 VERDICT
Next 1).  What train() runs on a ROCm device is vss_amd.minibatch.direct_minibatch: the one-launch row
gather with fp64 advantage sums (DirectRows.gather), the x6 GEMMs, the loss and output-layer backward
folded into the last hidden layer's launch, every gradient written into its FlatGrads view.  Here it is
compared with fp64 torch autograd of the reference's own loss (ppo_continuous_action_isaacgym.py:318-352 of
the reference: vss_amd.loss.reference_loss, the advantages normalised over the minibatch as ppo…:324-326),
next to torch's plain fp32 autograd of the same expressions:

* one GPU, rollout data (test_direct_minibatch_gradients_on_rollout_data_at_fp32_error_gpu): 4,096 fields x
  512 SA env steps = 2,097,152 rows; a 131,040-row minibatch (the reference's 4,095 envs: padded to 131,072)
  and the 2,097,152-row config-3 minibatch; the fused loss on and off;
* two ranks (test_direct_path_data_parallel_matches_hand_averaged_reference_gpu): ppo_update with the
  captured direct minibatch, FlatAdam and --norm-adv over both ranks' rows (gloo on the one GPU), against a
  single process that averages the two ranks' gradients by hand with the advantages normalised over the
  union of the ranks' minibatch rows -- in fp64 and fp32 -- and against the per-rank (local) normalisation,
  which the test must tell apart.
"""
import copy
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from test_ppo import _args, _free_port, make_agent
from vss_amd import minibatch as MB
from vss_amd.flat import FlatGrads
from vss_amd.loss import reference_loss

COEF = dict(clip_coef=0.2, ent_coef=0.005, vf_coef=4.0, clip_vloss=False)  # the reference's defaults
HERE = os.path.dirname(os.path.abspath(__file__))


def make_rollout_rows():
    """(agent, obs, act, logp_old, adv, ret, val): 2,097,152 rows of observations from 512 steps of the fused
    SA env at 4,096 fields under random actions, actions drawn from the Agent's policy, old log-probs within
    ~0.1 of the current ones (ratios around 1, some clipped), RAW advantages (mean 0.7, std 2.5: the
    normalisation matters), returns near the values."""
    from envs.vss import VSS, default_cfg
    from envs.wrappers import SingleAgent
    n, T = 4096, 512
    env = VSS(default_cfg(n), "cuda:0", "cuda:0", 0, True, False, False)
    W = SingleAgent(env)
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.empty(T * n, 52, device="cuda")
    o = W.reset()["obs"]
    for t in range(T):
        x[t * n:(t + 1) * n].copy_(o)
        o = W.step(torch.rand((n, 2), device="cuda", generator=g) * 2 - 1)[0]["obs"]
    agent = make_agent(2).cuda()
    with torch.no_grad():
        act, lp, _, v = agent.get_action_and_value(x)
    rows = x.shape[0]
    logp_old = lp + torch.randn(rows, device="cuda", generator=g) * 0.1
    adv = torch.randn(rows, device="cuda", generator=g) * 2.5 + 0.7
    ret = v.view(-1) + torch.randn(rows, device="cuda", generator=g) * 0.5
    val = v.view(-1).clone()
    del env, W
    return agent, x, act.contiguous(), logp_old, adv, ret, val


@pytest.fixture(scope="module")
def rollout_rows():
    return make_rollout_rows()


_REF = {}


def _reference_grads(agent0, data, inds, dtype):
    """torch autograd of the reference's minibatch loss (ppo…:318-349), the advantages normalised over the
    minibatch with torch's own expression (ppo…:325-326), in `dtype`: (loss, gradients as fp64)."""
    ag = copy.deepcopy(agent0).to(dtype)
    x, act, lp, adv, ret, val = [t[inds].to(dtype) for t in data]
    a = (adv - adv.mean()) / (adv.std() + 1e-8)
    loss, _ = reference_loss(ag.actor_mean(x), ag.actor_logstd, ag.critic(x), act, lp, a, ret, val, **COEF)
    grads = [t.double() for t in torch.autograd.grad(loss, list(ag.parameters()))]
    return float(loss.detach()), grads


def _rel(a, b):
    return float((a - b).norm() / b.norm())


# The bound on the direct path's gradient error relative to torch's plain fp32 autograd, per minibatch size.  At
# the reference's 4,095-env minibatch (131,040 rows) the x6 path is ~0.66 x torch's error (the round-5 VERDICT's
# 1.25 x holds with margin).  At config 3's 2,097,152 rows it is 1.3-1.4 x overall and up to 1.7 x for a weight
# matrix, its bias vectors 20-60 x (3e-5..6e-5 relative): the bf16 matrix cores' accumulation floors the running
# fp32 sum when it is aligned to products of comparable or larger size (tools/mfma_rounding_probe.hip), a small
# negative bias per MFMA that grows like K^1.5 with the contraction length, while an unbiased error grows like
# K^0.5 -- the weight gradients contract over 65,536 rows per split and the bias gradients sum 2 M column entries.
# Keeping the hi.hi products in an accumulator of their own removes it (tools/x6_accum_probe.hip variants 2 / 6)
# but needs 64 more registers than two waves per SIMD leave.  torch's own fp32 error at 2 M rows
# reaches 1.85e-5 for a weight matrix on this data (profiles/r06k_pytest_gpu.log), hence the 5e-5 cap there.
BOUNDS = {131040: dict(overall=1.25, matrix=1.25, small_matrix=2.0, abs=1e-5, bias=3e-5),
          2097152: dict(overall=1.6, matrix=2.0, small_matrix=2.0, abs=5e-5, bias=1e-4)}


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("mb", [131040, 2097152])
def test_direct_minibatch_gradients_on_rollout_data_at_fp32_error_gpu(rollout_rows, mb, fused, monkeypatch):
    """direct_minibatch -- the path train() takes -- on a minibatch of rollout rows gathered by
    DirectRows.gather (RAW advantages, normalised in the loss from the gather's fp64 sums), against fp64 autograd
    of the reference's expressions, next to torch's plain fp32 autograd (hipBLASLt GEMMs, fp32 normalisation):
    the relative gradient error over the whole gradient and per weight matrix within BOUNDS[mb] x torch fp32's
    (a matrix whose fp32 error is below 1e-6: 2 x) and below BOUNDS[mb]["abs"]; every bias vector below
    BOUNDS[mb]["bias"]; the loss within 1.25 x torch fp32's error of the fp64 loss, or 1e-6 relative."""
    monkeypatch.setattr(MB, "FUSED_LOSS", fused)
    bound = BOUNDS[mb]
    agent0, *data = rollout_rows
    x, act, lp, adv, ret, val = data
    batch = x.shape[0]
    inds = torch.randperm(batch, device="cuda", generator=torch.Generator(device="cuda").manual_seed(mb))[:mb]
    args = _args(norm_adv=True, **COEF)
    agent = copy.deepcopy(agent0)
    flat = FlatGrads(agent)
    assert MB.direct_minibatch_ok(agent, args, flat)
    pad = MB.padding_rows(mb, "cuda")
    assert (mb + pad) % 256 == 0 and (pad == 0) == (mb == 2097152)
    assert MB.fused_loss_ok(agent, mb + pad) or not fused
    rows = MB.DirectRows(mb, mb + pad, 52, 2, "cuda")
    src = rows.gather(inds, x, act, lp, adv, ret, val, True)
    flat.flat.fill_(float("nan"))  # every gradient view must be written
    loss_d, _ = MB.direct_minibatch(agent, args, rows.obs, rows.act, rows.logp, rows.adv, *src, rows.ret, rows.val)
    g_d = [p.grad.double() for p in agent.parameters()]
    assert not any(bool(torch.isnan(t).any()) for t in g_d)
    del rows
    key = mb
    if key not in _REF:
        _REF.clear()
        _REF[key] = (_reference_grads(agent0, data, inds, torch.float32),
                     _reference_grads(agent0, data, inds, torch.float64))
        torch.cuda.empty_cache()
    (loss_t, g_t), (loss_64, g_64) = _REF[key]
    cat = lambda gs: torch.cat([t.reshape(-1) for t in gs])  # noqa: E731
    e_d, e_t = _rel(cat(g_d), cat(g_64)), _rel(cat(g_t), cat(g_64))
    table = {name: (_rel(a, c), _rel(b, c)) for (name, _), a, b, c in zip(agent.named_parameters(), g_d, g_t, g_64)}
    print(f"\nmb {mb} fused {fused}: overall {e_d:.3e} vs torch fp32 {e_t:.3e}; " +
          "; ".join(f"{n} {a:.2e}/{b:.2e}" for n, (a, b) in table.items()))
    assert e_d <= bound["overall"] * e_t and e_d < bound["abs"], (e_d, e_t)
    for (name, p) in agent.named_parameters():
        ea, eb = table[name]
        if p.dim() == 2:
            assert ea <= (bound["matrix"] if eb >= 1e-6 else bound["small_matrix"]) * eb + 1e-9 and ea < bound["abs"], \
                (name, ea, eb)
        else:
            assert ea < bound["bias"], (name, ea, eb)
    assert abs(float(loss_d) - loss_64) <= max(1.25 * abs(loss_t - loss_64), 1e-6 * abs(loss_64)), \
        (float(loss_d), loss_t, loss_64)


# ---- data parallel: two ranks on the direct path ---------------------------------------------------------

DP_N = 32760          # rows per rank: 2 minibatches of 16,380 rows, each padded to 16,384 (64 x 256)
DP_EPOCHS = 3         # 6 minibatches: eager, capture, replays


def dp_rank_batch(rank: int, n: int = DP_N):
    """Rank `rank`'s rollout batch (CPU tensors): obs, act, logp_old, adv, ret, val.  The ranks' advantages
    come from different distributions (rank 0: N(0, 1), rank 1: N(2, 3^2)), so normalising over the union
    of both ranks' rows and normalising per rank give clearly different updates."""
    g = torch.Generator().manual_seed(100 + rank)
    obs = torch.randn(n, 52, generator=g)
    act = torch.randn(n, 2, generator=g) * 0.5
    logp = torch.randn(n, generator=g) * 0.1 - 2.0
    adv = torch.randn(n, generator=g) * (1.0 + 2.0 * rank) + 2.0 * rank
    ret = torch.randn(n, generator=g)
    val = torch.randn(n, generator=g)
    return obs, act, logp, adv, ret, val


def _dp_reference(adv_norm: str, dtype, world: int = 2):
    """A single process stepping one Agent with the hand-averaged gradients of `world` ranks (each rank's
    minibatch through torch autograd of the reference's loss, the permutation each rank's generator draws,
    EpochPermutations), clip_grad_norm_ and torch's Adam: the reference's loop (ppo…:306-354) run once
    over the union of the ranks' minibatches.  adv_norm "global": the advantages normalised with the mean /
    unbiased std of the union of the ranks' minibatch rows; "local": each rank's own."""
    agent = make_agent(2).cuda().to(dtype)
    opt = torch.optim.Adam(agent.parameters(), lr=1e-3, eps=1e-5)
    data = [[t.cuda().to(dtype) for t in dp_rank_batch(r)] for r in range(world)]
    perms = [MB.EpochPermutations(DP_N, "cuda", torch.Generator(device="cuda").manual_seed(7 + r), DP_EPOCHS)
             for r in range(world)]
    mb = DP_N // 2
    params = list(agent.parameters())
    for _ in range(DP_EPOCHS):
        p = [pm.next() for pm in perms]
        for start in range(0, DP_N, mb):
            inds = [p[r][start:start + mb] for r in range(world)]
            union = torch.cat([data[r][3][inds[r]] for r in range(world)])
            total = None
            for r in range(world):
                obs, act, logp, adv, ret, val = [t[inds[r]] for t in data[r]]
                if adv_norm == "global":
                    a = (adv - union.mean()) / (union.std() + 1e-8)
                else:
                    a = (adv - adv.mean()) / (adv.std() + 1e-8)
                loss, _ = reference_loss(agent.actor_mean(obs), agent.actor_logstd, agent.critic(obs), act, logp, a,
                                         ret, val, **COEF)
                g = torch.autograd.grad(loss, params)
                total = list(g) if total is None else [u + v for u, v in zip(total, g)]
            for prm, t in zip(params, total):
                prm.grad = t / world
            torch.nn.utils.clip_grad_norm_(params, 1.5)
            opt.step()
    return torch.cat([t.detach().double().reshape(-1) for t in params]).cpu()


@pytest.mark.gpu
def test_direct_path_data_parallel_matches_hand_averaged_reference_gpu(tmp_path):
    """Two ranks (torch.distributed.run, gloo, both on the one GPU) run ppo_update as train() does: the
    captured direct minibatch (MinibatchGraph.run_direct: DirectRows.gather's fp64 advantage sums all-reduced,
    adv_count = mb x world), FlatGrads' gradient all-reduce, FlatAdam.  Both ranks end with the same bits, and
    their weights match the hand-averaged single-process reference with union-normalised advantages:
    the distance of the update (w - w0) from the fp64 reference is at most 3 x that of the same reference in
    fp32 (+1e-6 relative), while the per-rank normalisation lies 100 x further away than that."""
    out = str(tmp_path)
    env = dict(os.environ, VSS_LOCAL_DEVICE="0", VSS_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(HERE, "dp_direct_worker.py"), out], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    w = [torch.load(os.path.join(out, f"w{k}.pt"), weights_only=True) for k in range(2)]
    assert torch.equal(w[0], w[1])
    info = [open(os.path.join(out, f"info{k}.txt")).read() for k in range(2)]
    assert all("direct=1 graph=1 replays=" in s for s in info), info
    w0 = torch.cat([t.detach().double().reshape(-1) for t in make_agent(2).parameters()])
    w_dp = w[0].double()
    ref64 = _dp_reference("global", torch.float64)
    ref32 = _dp_reference("global", torch.float32)
    loc64 = _dp_reference("local", torch.float64)
    step = (ref64 - w0).norm()
    d_dp = float((w_dp - ref64).norm() / step)
    d_32 = float((ref32 - ref64).norm() / step)
    d_loc = float((loc64 - ref64).norm() / step)
    assert d_dp <= 3.0 * d_32 + 1e-6, (d_dp, d_32)
    assert d_loc >= 100.0 * max(d_dp, d_32), (d_loc, d_dp, d_32)
