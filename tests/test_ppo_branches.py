"""The reference PPO's non-default branches (ppo_continuous_action_isaacgym.py:251-253, 335-344,
356-365) against hand computations, on CPU: --anneal-lr, --clip-vloss, --adaptative-lr (including
the data-parallel form, where the KL estimate that drives it is averaged over ranks) and the
--target-kl epoch break."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import ppo_continuous_action_isaacgym as P
from test_ppo import _args, _free_port, _synthetic_batch, make_agent


# ------------------------------------------------------------------------------ --anneal-lr
def test_anneal_lr_schedule_hand_values():
    """frac = 1 - (update - 1) / num_updates; lr = frac * lr0 (ppo…:251-253)."""
    got = [P.annealed_lr(u, 4, 1e-3) for u in range(1, 5)]
    assert got == pytest.approx([1e-3, 7.5e-4, 5e-4, 2.5e-4], rel=1e-12)
    assert P.annealed_lr(1, 1, 0.01) == 0.01


# ------------------------------------------------------------------------------ --clip-vloss
def test_clipped_value_loss_hand_values():
    """Row 0: v = 0.1, R = 0, V_old = 1.0: unclipped 0.01; v clipped to V_old - 0.2 = 0.8 -> 0.64;
    max 0.64.  Row 1: v = 2.0, R = 1.0, V_old = 1.9: unclipped 1; clipped v = 2.0 -> 1; max 1.
    v_loss = 0.5 * mean(0.64, 1) = 0.41.  Unclipped form: 0.5 * mean(0.01, 1) = 0.2525."""
    v, R, V = torch.tensor([0.1, 2.0]), torch.tensor([0.0, 1.0]), torch.tensor([1.0, 1.9])
    assert float(P.value_loss(v, R, V, 0.2, True)) == pytest.approx(0.41, abs=1e-6)
    assert float(P.value_loss(v, R, V, 0.2, False)) == pytest.approx(0.2525, abs=1e-6)


def _hand_update(agent, opt, args, data, gen, kl_of=None, lr_trace=None):
    """The reference's minibatch loop (ppo…:298-365), written out independently of ppo_update."""
    obs, act, logp, adv, ret, val = data
    n = obs.shape[0]
    mb = n // args.num_minibatches
    epochs = 0
    for epoch in range(args.update_epochs):
        epochs += 1
        perm = torch.randperm(n, generator=gen)
        for start in range(0, n, mb):
            i = perm[start:start + mb]
            _, nl, ent, nv = agent.get_action_and_value(obs[i], act[i])
            logratio = nl - logp[i]
            ratio = logratio.exp()
            approx_kl = ((ratio - 1) - logratio).mean().detach()
            if kl_of is not None:
                approx_kl = kl_of(approx_kl)
            a = adv[i]
            if args.norm_adv:
                a = (a - a.mean()) / (a.std() + 1e-8)
            pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - args.clip_coef, 1 + args.clip_coef)).mean()
            nv = nv.view(-1)
            if args.clip_vloss:
                vu = (nv - ret[i]) ** 2
                vc = val[i] + torch.clamp(nv - val[i], -args.clip_coef, args.clip_coef)
                vl = 0.5 * torch.max(vu, (vc - ret[i]) ** 2).mean()
            else:
                vl = 0.5 * ((nv - ret[i]) ** 2).mean()
            loss = pg - args.ent_coef * ent.mean() + vl * args.vf_coef
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(agent.parameters(), args.max_grad_norm)
            opt.step()
            if args.adaptative_lr:
                lr = opt.param_groups[0]["lr"]
                k = float(approx_kl)
                if k > 2.0 * args.threshold_kl:
                    opt.param_groups[0]["lr"] = max(lr / 1.5, 1e-6)
                elif k < 0.5 * args.threshold_kl:
                    opt.param_groups[0]["lr"] = min(lr * 1.5, 1e-2)
                if lr_trace is not None:
                    lr_trace.append(opt.param_groups[0]["lr"])
        if args.target_kl is not None and float(approx_kl) > args.target_kl:
            break
    return epochs


def _flat_params(agent):
    return torch.cat([p.detach().reshape(-1) for p in agent.parameters()])


def _run_both(args, data, seed=7):
    """ppo_update and the hand loop from the same initial weights and permutation stream."""
    a1, a2 = make_agent(2), make_agent(2)
    a2.load_state_dict(a1.state_dict())
    o1 = torch.optim.Adam(a1.parameters(), lr=args.learning_rate, eps=1e-5)
    o2 = torch.optim.Adam(a2.parameters(), lr=args.learning_rate, eps=1e-5)
    flat = P.FlatGrads(a1)
    stats = P.ppo_update(a1, o1, flat, args, *[data[k] for k in (0, 2, 1, 3, 4, 5)],
                         gen=torch.Generator().manual_seed(seed))
    epochs = _hand_update(a2, o2, args, data, torch.Generator().manual_seed(seed))
    return (a1, o1, stats), (a2, o2, epochs)


def test_clip_vloss_update_matches_hand_loop_and_differs_from_unclipped():
    """With V_old far from the returns the clip is active: the update follows the clipped loss
    (ppo…:335-344) -- equal to the hand loop -- and ends elsewhere than the unclipped update."""
    obs, act, logp, adv, ret, val = _synthetic_batch(5)
    val = ret + 3.0 * torch.sign(torch.randn(ret.shape, generator=torch.Generator().manual_seed(1)))
    data = (obs, act, logp, adv, ret, val)
    (a1, _, s1), (a2, _, _) = _run_both(_args(clip_vloss=True), data)
    torch.testing.assert_close(_flat_params(a1), _flat_params(a2), rtol=1e-5, atol=1e-6)
    (b1, _, _), _ = _run_both(_args(clip_vloss=False), data)
    assert not torch.allclose(_flat_params(a1), _flat_params(b1), rtol=1e-4, atol=1e-5)


# ------------------------------------------------------------------------------ --adaptative-lr
@pytest.mark.parametrize("lr,kl,want", [
    (1e-3, 0.02, 1e-3 / 1.5),       # kl > 2 x 0.008
    (1e-3, 0.001, 1.5e-3),          # kl < 0.004
    (1e-3, 0.008, 1e-3),            # in between: unchanged
    (1.2e-6, 1.0, 1e-6),            # floor
    (9e-3, 0.0, 1e-2),              # cap
])
def test_adapted_lr_hand_values(lr, kl, want):
    assert P.adapted_lr(lr, kl, 0.008) == pytest.approx(want, rel=1e-12)


def test_adaptative_lr_update_matches_hand_loop():
    """One process: the lr after every minibatch follows the KL of that minibatch (ppo…:356-361)."""
    data = _synthetic_batch(9)
    args = _args(adaptative_lr=True, threshold_kl=0.002, num_minibatches=4, update_epochs=3)
    (a1, o1, _), (a2, o2, _) = _run_both(args, data)
    assert o1.param_groups[0]["lr"] == pytest.approx(o2.param_groups[0]["lr"], rel=1e-9)
    assert o1.param_groups[0]["lr"] != args.learning_rate
    torch.testing.assert_close(_flat_params(a1), _flat_params(a2), rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------------------ --target-kl
def test_target_kl_breaks_after_the_first_epoch():
    """target_kl = 0: the first epoch's last-minibatch KL exceeds it, so the epoch loop breaks after
    one epoch (ppo…:363-365) -- the same weights as a one-epoch update; a huge target never breaks."""
    data = _synthetic_batch(11)
    (a1, _, s1), (a2, _, e2) = _run_both(_args(target_kl=0.0, update_epochs=4), data)
    assert s1["epochs_run"] == 1 and e2 == 1
    (b1, _, t1), _ = _run_both(_args(update_epochs=1), data)
    torch.testing.assert_close(_flat_params(a1), _flat_params(b1), rtol=0, atol=0)
    torch.testing.assert_close(_flat_params(a1), _flat_params(a2), rtol=1e-5, atol=1e-6)
    (c1, _, u1), _ = _run_both(_args(target_kl=1e9, update_epochs=3), data)
    assert u1["epochs_run"] == 3


# ------------------------------------------------------------------------------ data parallel
def _branch_worker(rank, world, port, q, which):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    agent = make_agent(2)
    flat = P.FlatGrads(agent)
    opt = torch.optim.Adam(agent.parameters(), lr=1e-3, eps=1e-5)
    args = _branch_args(which)
    obs, act, logp, adv, ret, val = _synthetic_batch(200 + rank)
    stats = P.ppo_update(agent, opt, flat, args, obs, logp, act, adv, ret, val, world=world,
                         gen=torch.Generator().manual_seed(7))
    q.put((rank, _flat_params(agent).numpy(), opt.param_groups[0]["lr"], int(stats["epochs_run"])))
    torch.distributed.destroy_process_group()


def _branch_args(which):
    if which == "adaptative":
        return _args(norm_adv=False, adaptative_lr=True, threshold_kl=0.002, update_epochs=3)
    return _args(norm_adv=False, target_kl=0.004, update_epochs=6)


@pytest.mark.parametrize("which", ["adaptative", "target_kl"])
def test_kl_driven_branches_world2_average_the_kl(which):
    """Two ranks (gloo) with different local batches: the KL estimate that drives --adaptative-lr
    and --target-kl is all-reduced to the mean over ranks (ppo…:456-459 of this build), so both
    ranks take the same decisions -- identical lr, epochs and weights -- and those equal a hand
    loop that averages both ranks' gradients AND KL estimates."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_branch_worker, args=(r, 2, port, q, which)) for r in range(2)]
    for p in procs:
        p.start()
    out = {r: (w, lr, ep) for r, w, lr, ep in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]

    # hand loop: both ranks' minibatches in lock-step, gradients and KL averaged
    args = _branch_args(which)
    agents = [make_agent(2), make_agent(2)]
    agents[1].load_state_dict(agents[0].state_dict())
    flats = [P.FlatGrads(a) for a in agents]
    opt = torch.optim.Adam(agents[0].parameters(), lr=1e-3, eps=1e-5)
    data = [_synthetic_batch(200 + r) for r in range(2)]
    gens = [torch.Generator().manual_seed(7) for _ in range(2)]
    n, mb = 256, 128
    epochs = 0
    for epoch in range(args.update_epochs):
        epochs += 1
        perms = [torch.randperm(n, generator=g) for g in gens]
        for start in range(0, n, mb):
            kls = []
            for r in range(2):
                obs, act, logp, adv, ret, val = data[r]
                i = perms[r][start:start + mb]
                _, nl, ent, nv = agents[r].get_action_and_value(obs[i], act[i])
                logratio = nl - logp[i]
                ratio = logratio.exp()
                kls.append(float(((ratio - 1) - logratio).mean().detach()))
                a = adv[i]
                pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 0.8, 1.2)).mean()
                vl = 0.5 * ((nv.view(-1) - ret[i]) ** 2).mean()
                flats[r].zero()
                (pg - args.ent_coef * ent.mean() + vl * args.vf_coef).backward()
            flats[0].flat.copy_((flats[0].flat + flats[1].flat) / 2)
            torch.nn.utils.clip_grad_norm_(agents[0].parameters(), args.max_grad_norm)
            opt.step()
            agents[1].load_state_dict(agents[0].state_dict())
            kl = (kls[0] + kls[1]) / 2
            if args.adaptative_lr:
                opt.param_groups[0]["lr"] = P.adapted_lr(opt.param_groups[0]["lr"], kl, args.threshold_kl)
        if args.target_kl is not None and kl > args.target_kl:
            break
    assert out[0][2] == epochs
    assert out[0][1] == pytest.approx(opt.param_groups[0]["lr"], rel=1e-9)
    np.testing.assert_allclose(out[0][0], _flat_params(agents[0]).numpy(), rtol=1e-5, atol=1e-6)
    if which == "target_kl":
        assert 1 <= epochs < args.update_epochs, "the KL break must fire inside the epoch loop"
    else:
        assert out[0][1] != 1e-3
