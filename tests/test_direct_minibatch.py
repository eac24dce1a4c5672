"""The update's minibatch without autograd (ppo_continuous_action_isaacgym.py direct_minibatch, round 5):
its three new launches -- the one-launch row gather with the advantages' fp64 sums
(vss_minibatch_gather), the loss from the output layers' epilogue parts with the advantage normalisation
and the output biases' gradients inside (vss_ppo_loss_direct), the output layer's backward without padded
copies (vss_output_backward_direct) -- each against its torch / autograd-path counterpart, and the whole
direct minibatch against the autograd path (minibatch_losses + FlatGrads.zeroed_backward, which the
CPU suite and the other shapes keep)."""
import numpy as np
import pytest
import torch

import ppo_continuous_action_isaacgym as P
from vss_amd import minibatch as MB
from vss_amd.update import sum_parts
from test_ppo import _args, _synthetic_batch, make_agent
from vss_amd.loss import (N_ACT, adv_part_sum, minibatch_gather, minibatch_gather_parts, ppo_loss, ppo_loss_direct,
                          ppo_loss_fused_finish, randperm)
from vss_amd.update import (linear_tanh_loss_x6, linear_tanh_loss_x6_ok, linear_tanh_out_x6, output_backward,
                            output_backward_direct, output_backward_direct_ok)


def test_direct_shapes_cpu():
    """The shapes the direct launches take, and the gather's part count (host-side, no GPU)."""
    assert all(output_backward_direct_ok(k, 256) for k in (1, 2, 3, 4, 6, 8))
    assert not output_backward_direct_ok(5, 256) and not output_backward_direct_ok(2, 384)
    assert minibatch_gather_parts(1) == 1 and minibatch_gather_parts(131040) == 256
    assert N_ACT == (1, 2, 3, 4, 6, 8)


def test_fused_loss_shapes_cpu():
    """The fused loss launch's shapes: a 256-wide last hidden layer on the x6 rows, 1 or 2 outputs
    (6 actions keep the separate launches)."""
    assert linear_tanh_loss_x6_ok(131072, 256, 256, 2) and linear_tanh_loss_x6_ok(256, 256, 256, 1)
    assert not linear_tanh_loss_x6_ok(131072, 256, 256, 6) and not linear_tanh_loss_x6_ok(131040, 256, 256, 2)
    assert not linear_tanh_loss_x6_ok(4096, 256, 512, 2)


def test_fused_loss_and_randperm_refuse_cpu_inputs_cpu():
    """No CPU fallback: the fused loss launch, its finish and vss_randperm refuse CPU tensors (and bad
    shapes) before touching the library."""
    x, w, b = torch.zeros(256, 256), torch.zeros(256, 256), torch.zeros(256)
    wo, bo = torch.zeros(2, 256), torch.zeros(2)
    with pytest.raises(ValueError):
        linear_tanh_loss_x6(x, w, b, wo, bo, 256, True)
    with pytest.raises(ValueError):  # 6 outputs: outside the fused shapes
        linear_tanh_loss_x6(x, w, b, torch.zeros(6, 256), torch.zeros(6), 256, True)
    for gvb in (torch.zeros(1), torch.zeros(3)):  # CPU tensors; a bad shape
        with pytest.raises(ValueError):
            ppo_loss_fused_finish(torch.zeros(4, 32), torch.zeros(4, 32), 256, torch.zeros(1, 2), 0.0, 0.5,
                                  torch.zeros(1, 2), torch.zeros(2), gvb)
    with pytest.raises(ValueError):
        randperm(10, torch.zeros(1, dtype=torch.int64))
    with pytest.raises(ValueError):  # key bits outside [1, 32]
        randperm(10, torch.zeros(1, dtype=torch.int64), key_bits=33)


def test_direct_minibatch_not_for_cpu_or_amp():
    """direct_minibatch_ok: FlatGrads-owned GPU gradients, fp32 networks -- CPU agents and --amp keep the
    autograd path."""
    agent = make_agent(2)
    flat = P.FlatGrads(agent)
    assert not P.direct_minibatch_ok(agent, _args(), flat)  # CPU gradients
    assert not P.direct_minibatch_ok(agent, _args(), None)
    assert not P.direct_minibatch_ok(agent, _args(amp="bf16"), flat)


@pytest.mark.gpu
@pytest.mark.parametrize("mb,rows_pad,obs_w", [(1000, 1024, 52), (131040, 131072, 52), (300, 512, 7)])
def test_minibatch_gather_matches_index_select_gpu(mb, rows_pad, obs_w):
    """vss_minibatch_gather = index_select of every batch tensor (the padding rows repeating the
    minibatch's rows), bit for bit; the advantages' parts sum to their fp64 sum and sum of squares; an
    index outside the batch gathers NaN (no out-of-bounds read)."""
    batch = 3 * mb + 17
    g = torch.Generator(device="cuda").manual_seed(1)
    b_obs = torch.randn(batch, obs_w, device="cuda", generator=g)
    b_act = torch.randn(batch, 2, device="cuda", generator=g)
    b_s = [torch.randn(batch, device="cuda", generator=g) for _ in range(4)]
    inds = torch.randperm(batch, device="cuda", generator=g)[:mb].contiguous()
    z = lambda *s, dt=torch.float32: torch.full(s, 5.0, device="cuda", dtype=dt)  # noqa: E731
    obs, act, outs = z(rows_pad, obs_w), z(rows_pad, 2), [z(mb) for _ in range(4)]
    part = z(minibatch_gather_parts(mb), 2, dt=torch.float64)
    minibatch_gather(inds, b_obs, b_act, *b_s, obs, act, *outs, part)
    pad_inds = torch.cat([inds, inds.repeat(rows_pad // mb + 1)[:rows_pad - mb]])
    assert torch.equal(obs, b_obs[pad_inds]) and torch.equal(act, b_act[pad_inds])
    for o, b in zip(outs, b_s):
        assert torch.equal(o, b[inds])
    a = b_s[1][inds].double()  # the advantages (logp, adv, ret, val order)
    tot = adv_part_sum(part, torch.empty(1, 2, device="cuda", dtype=torch.float64))
    np.testing.assert_allclose(tot.cpu().numpy()[0], [float(a.sum()), float((a * a).sum())], rtol=1e-12, atol=1e-9)
    bad = inds.clone()
    bad[3] = batch + 5
    minibatch_gather(bad, b_obs, b_act, *b_s, obs, act, *outs, part)
    assert torch.isnan(obs[3]).all() and torch.isnan(outs[0][3]) and not torch.isnan(obs[4]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("k_out", [1, 2, 6])
def test_output_backward_direct_matches_padded_pass_gpu(k_out):
    """vss_output_backward_direct (g_out and w_out as they are, <= 256 parts) = vss_output_backward on the
    zero-padded copies: the same gradient bits (the padding adds exact zeros), the bias and weight
    gradients within fp32 summation-order rounding."""
    rows, n = 131072, 256
    g = torch.Generator(device="cuda").manual_seed(2)
    go = torch.randn(rows, k_out, device="cuda", generator=g) * 1e-3
    w = torch.randn(k_out, n, device="cuda", generator=g) / 16
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    gz0, db0, dw0 = output_backward(go, w, y)
    defer = []
    gz1, db1, dw1 = output_backward_direct(go, w, y, defer=defer)
    assert len(defer) == 2 and all(p.shape[0] <= 256 for p, _ in defer)
    sum_parts(defer)
    assert torch.equal(gz0, gz1)
    ref_db, ref_dw = (go.double() @ w.double() * (1 - y.double() ** 2)).sum(0), go.double().t() @ y.double()
    for got, want in ((db0, ref_db), (db1, ref_db), (dw0, ref_dw), (dw1, ref_dw)):
        assert float((got.double() - want).abs().max()) <= 1e-5 * float(want.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("norm,clip_vloss", [(True, False), (True, True), (False, True)])
def test_ppo_loss_direct_matches_loss_on_summed_outputs_gpu(norm, clip_vloss):
    """vss_ppo_loss_direct on the epilogue parts + biases and the RAW advantages = vss_ppo_loss on the
    summed outputs and the advantages normalised with the same fp64 statistics: the same losses, row
    gradients and log-std gradient; the output biases' gradients = the row gradients' column sums."""
    rows, rows_pad, n_act = 131040, 131072, 2
    g = torch.Generator(device="cuda").manual_seed(3)
    mp = torch.randn(4, rows_pad, n_act, device="cuda", generator=g) * 0.1
    vp = torch.randn(4, rows_pad, 1, device="cuda", generator=g)
    bm, bv = torch.randn(n_act, device="cuda", generator=g) * 0.1, torch.randn(1, device="cuda", generator=g)
    logstd = torch.randn(1, n_act, device="cuda", generator=g) * 0.1
    act = torch.randn(rows_pad, n_act, device="cuda", generator=g) * 0.3
    logp, adv, ret, val = [torch.randn(rows, device="cuda", generator=g) for _ in range(4)]
    logp = logp - 1.0
    part = None
    if norm:
        a = adv.double()
        part = torch.stack([a.sum(), (a * a).sum()]).view(1, 2).contiguous()
        m = part[0, 0] / rows
        sd = ((part[0, 1] - rows * m * m) / (rows - 1)).clamp(min=0).sqrt()
        adv_n = (adv - m.float()) / (sd.float() + 1e-8)
    else:
        adv_n = adv
    mean = mp.sum(0) + bm
    value = vp.sum(0) + bv
    loss0, st0 = ppo_loss(mean.requires_grad_(), logstd.requires_grad_(), value.requires_grad_(), act, logp, adv_n,
                          ret, val, 0.2, 0.01, 0.5, clip_vloss)
    loss0.backward()
    gl, dbm, dbv = torch.empty_like(logstd), torch.empty(n_act, device="cuda"), torch.empty(1, device="cuda")
    gm, gv, loss1, st1 = ppo_loss_direct(mp, bm, vp, bv, logstd.detach(), act, logp, adv, part, rows, ret, val,
                                         0.2, 0.01, 0.5, clip_vloss, gl, dbm, dbv)
    torch.testing.assert_close(loss1, loss0.detach(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(st1, torch.stack([t.detach() for t in st0]), rtol=2e-6, atol=1e-7)
    scale_m, scale_v = float(mean.grad.abs().max()), float(value.grad.abs().max())
    assert float((gm - mean.grad).abs().max()) <= 1e-5 * scale_m
    assert float((gv - value.grad).abs().max()) <= 1e-5 * scale_v
    torch.testing.assert_close(gl, logstd.grad, rtol=1e-5, atol=1e-7)
    assert float((dbm.double() - gm.double().sum(0)).abs().max()) <= 1e-6 * float(gm.double().abs().sum())
    assert float((dbv.double() - gv.double().sum()).abs().max()) <= 1e-6 * float(gv.double().abs().sum())


@pytest.mark.gpu
@pytest.mark.parametrize("rows,rows_pad,n_act,norm,clip_vloss", [
    (131040, 131072, 2, True, False), (65536, 65536, 2, True, True), (1000, 1024, 1, False, True),
    (300, 512, 2, True, True), (1, 256, 1, False, False)])
def test_fused_loss_matches_separate_launches_gpu(rows, rows_pad, n_act, norm, clip_vloss):
    """vss_linear_tanh_loss_bf16x6 (actor and critic) + vss_ppo_loss_fused_finish = the separate launches
    direct_minibatch otherwise runs (vss_linear_tanh_out_bf16x6 with parts, vss_ppo_loss_direct,
    vss_output_backward_direct): the hidden layer's gradient, its bias and the output weight's gradients,
    the loss, its statistics and the log-std / output-bias gradients within fp32 summation-order rounding;
    the padding rows' gradient exactly zero."""
    g = torch.Generator(device="cuda").manual_seed(7)
    rn = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    xa, xc = torch.tanh(rn(rows_pad, 256)), torch.tanh(rn(rows_pad, 256))
    wa, wc = rn(256, 256) / 16, rn(256, 256) / 16
    ba, bc = rn(256) * 0.1, rn(256) * 0.1
    woa, woc = rn(n_act, 256) / 16, rn(1, 256) / 16
    boa, boc = rn(n_act) * 0.1, rn(1)
    logstd = rn(1, n_act) * 0.1
    act = rn(rows_pad, n_act) * 0.3
    logp, adv, ret, val = rn(rows) - 1.0, rn(rows), rn(rows), rn(rows)
    part = None
    if norm:
        a = adv.double()
        part = torch.stack([a.sum(), (a * a).sum()]).view(1, 2).contiguous()
    kw = dict(clip_coef=0.2, vf_coef=0.5, clip_vloss=clip_vloss)
    # the separate launches
    ya, pa = linear_tanh_out_x6(xa, wa, ba, woa, boa, parts=True)
    yc, pc = linear_tanh_out_x6(xc, wc, bc, woc, boc, parts=True)
    gl0, dbm0, dbv0 = torch.empty_like(logstd), torch.empty(n_act, device="cuda"), torch.empty(1, device="cuda")
    gm, gv, loss0, st0 = ppo_loss_direct(pa, boa, pc, boc, logstd, act, logp, adv, part, rows, ret, val, 0.2, 0.01, 0.5,
                                         clip_vloss, gl0, dbm0, dbv0)
    ref = [output_backward_direct(gm, woa, ya), output_backward_direct(gv, woc, yc)]
    # the fused launches
    gl1, dbm1, dbv1 = torch.empty_like(logstd), torch.empty(n_act, device="cuda"), torch.empty(1, device="cuda")
    fa = linear_tanh_loss_x6(xa, wa, ba, woa, boa, rows, True, act=act, logp=logp, adv=adv, adv_part=part,
                             adv_count=rows, logstd=logstd, **kw)
    fc = linear_tanh_loss_x6(xc, wc, bc, woc, boc, rows, False, ret=ret, val=val, **kw)
    loss1, st1 = ppo_loss_fused_finish(fa[3], fc[3], rows, logstd, 0.01, 0.5, gl1, dbm1, dbv1)
    for (gz0, db0, dw0), (gz1, db1, dw1, _) in zip(ref, (fa, fc)):
        assert torch.equal(gz1[rows:], torch.zeros_like(gz1[rows:]))
        for got, want in ((gz1, gz0), (db1, db0), (dw1, dw0)):
            assert float((got - want).abs().max()) <= 2e-5 * float(want.abs().max()), (got.shape, want.shape)
    torch.testing.assert_close(loss1, loss0, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(st1, st0, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(gl1, gl0, rtol=2e-5, atol=1e-6)
    for got, want in ((dbm1, dbm0), (dbv1, dbv0)):
        assert float((got - want).abs().max()) <= 2e-5 * max(float(want.abs().max()), 1e-3)


def _grads(agent):
    return [p.grad.detach().clone() for p in agent.parameters()]


@pytest.mark.gpu
@pytest.mark.parametrize("n,nmb,act_dim,norm_adv,clip_vloss,fused", [
    (262080, 2, 2, True, False, True),   # 131,040-row minibatches (4,095 envs): 32 padding rows
    (262080, 2, 2, True, False, False), (32768, 2, 2, True, True, True), (32768, 2, 1, False, True, True),
    (32768, 4, 6, False, True, True), (4096, 2, 2, True, False, True)])
def test_direct_minibatch_matches_autograd_path_gpu(n, nmb, act_dim, norm_adv, clip_vloss, fused, monkeypatch):
    """One minibatch through direct_minibatch (gather, forward, loss, backward into the FlatGrads views)
    against the autograd path on the same rows (index_select + normalize_advantages + minibatch_losses +
    zeroed_backward): every parameter's gradient within 2e-5 of its largest entry, the statistics within
    fp32 rounding; every gradient view written (the flat buffer starts as NaN)."""
    monkeypatch.setattr(MB, "FUSED_LOSS", fused)  # the loss in the last hidden layers' launches, or apart
    args = _args(norm_adv=norm_adv, clip_vloss=clip_vloss, num_minibatches=nmb)
    g = torch.Generator().manual_seed(11)
    obs, _, logp, adv, ret, val = [t.cuda() for t in _synthetic_batch(5, n)]
    act = (torch.randn(n, act_dim, generator=g) * 0.5).cuda()
    agent = make_agent(act_dim).cuda()
    flat = P.FlatGrads(agent)
    assert P.direct_minibatch_ok(agent, args, flat)
    mb = n // nmb
    inds = torch.randperm(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(4))[:mb]
    pad = P.padding_rows(mb, "cuda")
    inds_pad = torch.cat([inds, inds.repeat(-(-pad // mb))[:pad]]) if pad else inds
    mb_adv = P.normalize_advantages(adv[inds]) if norm_adv else adv[inds]
    loss, st0 = P.minibatch_losses(agent, args, obs[inds_pad], act[inds_pad], logp[inds], mb_adv, ret[inds], val[inds])
    flat.zeroed_backward(loss)
    want = _grads(agent)
    flat.flat.fill_(float("nan"))
    rows = P.DirectRows(mb, mb + pad, 52, act_dim, "cuda")
    src = rows.gather(inds, obs, act, logp, adv, ret, val, norm_adv)
    _, st1 = P.direct_minibatch(agent, args, rows.obs, rows.act, rows.logp, rows.adv, *src, rows.ret, rows.val)
    got = _grads(agent)
    for (name, _), a, b in zip(agent.named_parameters(), want, got):
        assert not torch.isnan(b).any(), name
        assert float((a - b).abs().max()) <= 2e-5 * float(a.abs().max()) + 1e-12, name
    for a, b in zip(st0, st1):
        assert abs(float(a) - float(b)) <= 2e-5 * max(abs(float(a)), 1e-3)
    # the same minibatch again: the same bits (no atomics, fixed orders)
    _, st2 = P.direct_minibatch(agent, args, rows.obs, rows.act, rows.logp, rows.adv, *src, rows.ret, rows.val)
    assert all(torch.equal(a, b) for a, b in zip(got, _grads(agent)))
    assert all(float(a) == float(b) for a, b in zip(st1, st2))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 1000, 262080, 8388608])
def test_randperm_is_a_seeded_permutation_gpu(n):
    """vss_randperm: a permutation of [0, n) (sorted = arange), the same for the same seed, different
    for another; at 8,388,608 (the SA batch) the scratch and the 4-pass sort hold."""
    dev = "cuda"
    s1 = torch.tensor([1234567], dtype=torch.int64, device=dev)
    s2 = torch.tensor([-987654321], dtype=torch.int64, device=dev)
    p1, p1b, p2 = randperm(n, s1), randperm(n, s1), randperm(n, s2)
    assert p1.dtype == torch.int64 and p1.shape == (n,)
    assert torch.equal(torch.sort(p1).values, torch.arange(n, device=dev))
    assert torch.equal(p1, p1b)
    if n >= 1000:
        assert not torch.equal(p1, p2) and not torch.equal(p1, torch.arange(n, device=dev))


@pytest.mark.gpu
@pytest.mark.parametrize("key_bits", [32, 2, 1])
def test_randperm_is_uniform_gpu(key_bits):
    """Uniformity of vss_randperm over seeds: for n = 8, 10,000 seeds, every (element, position) count
    within 5 sigma of 1,250, and the fixed-point count's mean near 1 (a uniform permutation's).  With 2 or 1
    random key bits per index (4 or 2 key values for 8 indices) nearly every key is tied, so the result is
    uniform only if the sort's tied runs are shuffled: a stable sort alone would keep them in index order."""
    n, draws = 8, 10000
    seeds = torch.randint(-2 ** 62, 2 ** 62, (draws,), generator=torch.Generator().manual_seed(5 + key_bits))
    counts = torch.zeros(n, n, dtype=torch.int64)
    fixed = 0
    for s in seeds.tolist():
        p = randperm(n, torch.tensor([s], dtype=torch.int64, device="cuda"), key_bits=key_bits).cpu()
        counts[torch.arange(n), p] += 1
        fixed += int((p == torch.arange(n)).sum())
    expect = draws / n
    sigma = (draws * (1 / n) * (1 - 1 / n)) ** 0.5
    assert float((counts.double() - expect).abs().max()) < 5 * sigma, counts
    assert abs(fixed / draws - 1.0) < 0.05


def _splitmix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


@pytest.mark.gpu
def test_randperm_ties_are_shuffled_at_batch_size_gpu():
    """At the SA batch (8,388,608 indices, 32 random bits each) ~n^2 / 2^33 = 8,192 adjacent pairs of the
    permutation carry tied random bits.  Recomputing every index's bits on the host (splitmix64 of seed and
    index, as csrc/vss_loss.hip) from the permutation: the bits are sorted (non-decreasing), about the expected
    number of tied pairs occur, and within tied pairs the lower index comes first half the time (a stable sort
    alone: every time), within 5 sigma."""
    n, seed = 8388608, 0x1234_5678_9ABC_DEF
    p = randperm(n, torch.tensor([seed], dtype=torch.int64, device="cuda")).cpu().numpy()
    assert np.array_equal(np.sort(p), np.arange(n))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        r = _splitmix64(np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(32)
    keys = r[p]
    assert bool(np.all(keys[1:] >= keys[:-1]))
    tied = np.nonzero(keys[1:] == keys[:-1])[0]
    expect = n * (n - 1) / 2 / 2 ** 32
    assert abs(len(tied) - expect) < 5 * expect ** 0.5, (len(tied), expect)
    ascending = float(np.mean(p[tied] < p[tied + 1]))
    assert abs(ascending - 0.5) < 5 * (0.25 / len(tied)) ** 0.5, ascending


@pytest.mark.gpu
@pytest.mark.parametrize("hip", [True, False])
def test_epoch_permutations_gpu(hip, monkeypatch):
    """EpochPermutations on the GPU (side stream, drawn one epoch ahead): every epoch a permutation of the
    batch, the same sequence for the same generator seed; without VSS_RANDPERM=hip (the default) exactly
    torch.randperm's sequence from that generator."""
    monkeypatch.setattr(MB, "RANDPERM_HIP", hip)
    batch, epochs = 100000, 4

    def draw(seed):
        gen = torch.Generator(device="cuda").manual_seed(seed)
        perms = P.EpochPermutations(batch, "cuda", gen, epochs)
        return [perms.next().clone() for _ in range(epochs)]

    a, b, c = draw(5), draw(5), draw(6)
    ar = torch.arange(batch, device="cuda")
    for p in a:
        assert torch.equal(torch.sort(p).values, ar)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert not torch.equal(a[0], c[0]) and not torch.equal(a[0], a[1])
    if not hip:
        gen = torch.Generator(device="cuda").manual_seed(5)
        want = [torch.randperm(batch, device="cuda", generator=gen) for _ in range(epochs)]
        assert all(torch.equal(x, y) for x, y in zip(a, want))
