"""The fused PPO minibatch loss (csrc/vss_loss.hip, vss_amd/loss.py) against autograd of the reference's
expressions (ppo_continuous_action_isaacgym.py:318-349, restated in vss_amd.loss.reference_loss) on the
same inputs: the loss, the six logged statistics and the gradients into the actor means, the log-std and
the critic values, with and without --clip-vloss, with normalised and raw advantages, for the SA/DMA
(2) and CMA (6) action widths, at the reference's default minibatch (4,095 envs x 128 / 4 = 131,040
rows) padded to whole 256-row tiles as the update pads it.  Tolerances (fp32 summation order): the
losses and statistics 2e-5 relative (clipfrac within 4 rows), the gradients 1e-4 relative to their
largest entry, and exactly zero for the padding rows."""
import pytest
import torch

from vss_amd.loss import ppo_loss, reference_loss


def _inputs(rows, pad, n_act, seed, dev, norm_adv):
    g = torch.Generator(device=dev).manual_seed(seed)
    R = rows + pad
    mean = (torch.randn(R, n_act, device=dev, generator=g) * 0.5).requires_grad_()
    logstd = (torch.randn(1, n_act, device=dev, generator=g) * 0.3).requires_grad_()
    value = torch.randn(R, 1, device=dev, generator=g).requires_grad_()
    action = (mean.detach() + torch.randn(R, n_act, device=dev, generator=g) * torch.exp(logstd.detach())).contiguous()
    with torch.no_grad():
        var = torch.exp(logstd) ** 2
        lp = (-((action - mean) ** 2) / (2 * var) - logstd - 0.9189385332046727).sum(1)[:rows]
    # old log-probs around the new ones: ratios spread over and beyond [1 - clip, 1 + clip]
    logp_old = lp + torch.randn(rows, device=dev, generator=g) * 0.25
    adv = torch.randn(rows, device=dev, generator=g) * 2.0 + 0.3
    if norm_adv:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ret = torch.randn(rows, device=dev, generator=g)
    val = value.detach()[:rows, 0] + torch.randn(rows, device=dev, generator=g) * 0.3
    return mean, logstd, value, action, logp_old, adv, ret, val


def test_ppo_loss_cpu_is_the_reference_expressions():
    """On CPU tensors ppo_loss IS the reference's torch expressions (the CPU suite's PPO loop)."""
    ins = _inputs(300, 0, 2, 1, "cpu", True)
    loss, st = ppo_loss(*ins, 0.2, 0.005, 4.0, False)
    loss.backward()
    g = [t.grad.clone() for t in ins[:3]]
    for t in ins[:3]:
        t.grad = None
    ref, rst = reference_loss(*ins, 0.2, 0.005, 4.0, False)
    ref.backward()
    assert float(loss.detach()) == float(ref.detach()) and all(float(a) == float(b) for a, b in zip(st, rst))
    assert all(torch.equal(a, t.grad) for a, t in zip(g, ins[:3]))


def test_ppo_loss_refuses_bad_shapes_cpu():
    ins = list(_inputs(64, 0, 2, 2, "cpu", False))
    ins[4] = ins[4][:10]  # logprob_old shorter than adv
    with pytest.raises(ValueError):
        ppo_loss(*ins, 0.2, 0.005, 4.0, False)


@pytest.mark.gpu
@pytest.mark.parametrize("n_act", [2, 6])
@pytest.mark.parametrize("clip_vloss", [False, True])
@pytest.mark.parametrize("norm_adv", [True, False])
def test_fused_loss_matches_reference_autograd_gpu(n_act, clip_vloss, norm_adv):
    _check_fused_loss(n_act, clip_vloss, norm_adv)


@pytest.mark.gpu
@pytest.mark.parametrize("n_act", [1, 3, 4, 8])
@pytest.mark.parametrize("clip_vloss", [False, True])
def test_fused_loss_other_action_widths_gpu(n_act, clip_vloss):
    """The other widths vss_ppo_loss is built for (N_ACT): the same checks as the Agent's 2 and 6."""
    _check_fused_loss(n_act, clip_vloss, True)


@pytest.mark.gpu
def test_fused_loss_refuses_inputs_the_kernel_would_misread_gpu():
    """Fewer action rows than network rows (the kernel would read past the buffer), or an input that is
    not fp32 on the networks' device (it would be reinterpreted as fp32 device memory): ValueError."""
    ins = list(_inputs(1000, 24, 2, 5, "cuda", True))
    bad = list(ins)
    bad[3] = ins[3][:1010]
    with pytest.raises(ValueError):
        ppo_loss(*bad, 0.2, 0.005, 4.0, False)
    for k in range(4, 8):
        for t in (ins[k].double(), ins[k].cpu()):
            bad = list(ins)
            bad[k] = t
            with pytest.raises(ValueError):
                ppo_loss(*bad, 0.2, 0.005, 4.0, False)


def _check_fused_loss(n_act, clip_vloss, norm_adv):
    rows, pad = 131040, 224
    ins = _inputs(rows, pad, n_act, 7 + n_act + 2 * clip_vloss, "cuda", norm_adv)
    coef = (0.2, 0.005, 4.0, clip_vloss)
    loss, st = ppo_loss(*ins, *coef)
    loss.backward()
    got = [t.grad.clone() for t in ins[:3]]
    for t in ins[:3]:
        t.grad = None
    ref, rst = reference_loss(*ins, *coef)
    ref.backward()
    want = [t.grad for t in ins[:3]]
    torch.testing.assert_close(loss, ref, rtol=2e-5, atol=1e-6)
    names = ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl")
    for name, a, b in zip(names, st[:5], rst[:5]):
        torch.testing.assert_close(a, b.detach(), rtol=2e-5, atol=1e-6, msg=name)
    assert abs(float(st[5]) - float(rst[5])) <= 4.0 / rows, (float(st[5]), float(rst[5]))
    assert 0.05 < float(rst[5]) < 0.95  # the case exercises both the clipped and the unclipped branch
    for name, a, b in zip(("mean", "logstd", "value"), got, want):
        scale = float(b.abs().max())
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * scale, msg=name)
    # the padding rows carry no gradient
    assert torch.count_nonzero(got[0][rows:]) == 0 and torch.count_nonzero(got[2][rows:]) == 0


@pytest.mark.gpu
def test_fused_loss_deterministic_gpu():
    """The partial sums are reduced in a fixed order: two calls give the same bits."""
    ins = _inputs(2097152, 0, 2, 3, "cuda", True)
    a = ppo_loss(*ins, 0.2, 0.005, 4.0, True)
    b = ppo_loss(*ins, 0.2, 0.005, 4.0, True)
    assert torch.equal(a[0], b[0]) and all(torch.equal(x, y) for x, y in zip(a[1], b[1]))
