"""PPO-update helpers (csrc/vss_update.hip): vss_tanh_grad_bias (one HIP pass for the backward of a
hidden tanh layer) against torch's tanh_backward + bias-gradient reduction (the fp32 reference of
the same op); the fused-epilogue GEMMs vss_linear_tanh / vss_linear_tanh_backward and the output
layer's one-pass backward vss_output_backward against torch fp32 and fp64; and the update's
gradients through either path against plain autograd."""
import pytest
import torch

import ppo_continuous_action_isaacgym as P
from vss_amd import mlp as M
from vss_amd import _native as N
from vss_amd.update import linear_tanh, linear_tanh_backward, output_backward, tanh_grad_bias

from test_ppo import make_agent


def test_cpu_formula_matches_autograd():
    g = torch.Generator().manual_seed(0)
    z = torch.randn(300, 256, generator=g, requires_grad=True)
    gy = torch.randn(300, 256, generator=g)
    y = torch.tanh(z)
    (ref,) = torch.autograd.grad(y, z, gy)
    gz, db = tanh_grad_bias(gy, y.detach())
    torch.testing.assert_close(gz, ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(db, ref.sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("cols", [64, 256, 512, 1024])
@pytest.mark.parametrize("rows", [0, 1, 3, 2047, 2048, 2049, 100_003])
def test_tanh_grad_bias_gpu(rows, cols):
    g = torch.Generator(device="cuda").manual_seed(rows * 7 + cols)
    y = torch.tanh(torch.randn(rows, cols, device="cuda", generator=g) * 2)
    gy = torch.randn(rows, cols, device="cuda", generator=g)
    gz, db = tanh_grad_bias(gy, y)
    ref = torch.ops.aten.tanh_backward(gy, y)  # what autograd of nn.Tanh issues
    # one fused multiply-add less rounding than torch's g * (1 - y*y): within 2 ulp
    torch.testing.assert_close(gz, ref, rtol=3e-7, atol=1e-30)
    torch.testing.assert_close(db, gz.sum(0), rtol=2e-5, atol=2e-5 * (rows ** 0.5 + 1))
    assert db.shape == (cols,)


@pytest.mark.gpu
def test_tanh_grad_bias_refusals_gpu():
    y = torch.zeros(8, 300, device="cuda")
    with pytest.raises(ValueError):
        tanh_grad_bias(y, y)  # width the kernel does not take
    lib = N.load()
    buf = torch.zeros(4 * 256 + 1, device="cuda")
    part = torch.zeros(256, device="cuda")
    mis = buf[1:].data_ptr()  # 4-B offset: not 16-B aligned
    assert lib.vss_tanh_grad_bias(N.stream_of(buf.device), 4, 256, mis, buf.data_ptr(), buf.data_ptr(),
                                  part.data_ptr()) != 0
    assert lib.vss_tanh_grad_bias(N.stream_of(buf.device), 4, 300, buf.data_ptr(), buf.data_ptr(),
                                  buf.data_ptr(), part.data_ptr()) != 0


def test_cpu_fused_layer_formulas_match_autograd():
    """The CPU forms of linear_tanh / linear_tanh_backward (what the CPU suite's PPO loop runs) are
    autograd's nn.Linear -> nn.Tanh -> nn.Linear chain."""
    g = torch.Generator().manual_seed(1)
    x = torch.randn(40, 52, generator=g)
    w0, b0 = torch.randn(256, 52, generator=g) * 0.1, torch.randn(256, generator=g) * 0.1
    w1 = (torch.randn(128, 256, generator=g) * 0.1).requires_grad_()
    gout = torch.randn(40, 128, generator=g)
    z0 = torch.addmm(b0, x, w0.t()).requires_grad_()
    y0 = torch.tanh(z0)
    (ref,) = torch.autograd.grad(y0.mm(w1.t()), z0, gout)
    torch.testing.assert_close(linear_tanh(x, w0, b0), y0.detach(), rtol=0, atol=0)
    gz, db = linear_tanh_backward(gout, w1.detach(), y0.detach())
    torch.testing.assert_close(gz, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(db, ref.sum(0), rtol=1e-5, atol=1e-5)


def test_update_mlp_path_cpu_matches_autograd():
    """The update's MLP node (_TanhMLP) on CPU tensors: the Agent's outputs and autograd's gradients."""
    agent = make_agent(2)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(96, 52, generator=g)
    a = torch.randn(96, 2, generator=g) * 0.5
    outs_ref = agent.get_action_and_value(x, a)
    grads_ref = torch.autograd.grad(outs_ref[1].sum() + outs_ref[2].sum() + outs_ref[3].sum(), list(agent.parameters()))
    outs = P.get_action_and_value_update(agent, x, a)
    for u, v in zip(outs[1:], outs_ref[1:]):
        torch.testing.assert_close(u, v, rtol=1e-6, atol=1e-6)
    grads = torch.autograd.grad(outs[1].sum() + outs[2].sum() + outs[3].sum(), list(agent.parameters()))
    for (name, _), u, v in zip(agent.named_parameters(), grads, grads_ref):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-4 * float(v.abs().max()) + 1e-7, msg=name)


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(52, 256), (256, 512), (512, 512), (512, 256), (8, 128), (56, 256), (64, 256)])
@pytest.mark.parametrize("rows", [1, 127, 129, 4133, 70_000, 65_536])  # 65,536: exact shape, 4+ tiles per block
def test_linear_tanh_gpu(rows, k, n):
    """vss_linear_tanh vs the fp32 torch op (addmm + tanh) and an fp64 reference: the fused GEMM
    sums in a different order and its tanh is within a few ulp, so within fp32 GEMM rounding."""
    g = torch.Generator(device="cuda").manual_seed(rows + 7 * k + n)
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) * (2.0 / k) ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    y = linear_tanh(x, w, b)
    ref64 = torch.tanh(x.double() @ w.double().t() + b.double())
    ref32 = torch.addmm(b, x, w.t()).tanh_()
    # fp32 GEMM error bound ~ k * eps * sum|x w| (sum|x w| <= sqrt(2k) here) + a few ulp of tanh
    tol = 4e-7 * (k * (2.0 * k) ** 0.5) ** 0.5 + 1e-6
    assert float((y.double() - ref64).abs().max()) < tol
    assert float((y - ref32).abs().max()) < 2 * tol
    assert y.shape == (rows, n) and bool(torch.isfinite(y).all())


@pytest.mark.gpu
def test_linear_tanh_small_arguments_keep_relative_precision_gpu():
    """The tanh epilogue keeps relative precision near 0 (odd polynomial for |z| < 0.3, where the
    exponential form would cancel) and saturates cleanly at large |z|."""
    z = torch.cat([torch.logspace(-30, 1.5, 20000, device="cuda"), torch.tensor([0.0, 9.0, 20.0, 88.0], device="cuda")])
    z = torch.cat([z, -z])
    rows = z.numel()
    x = torch.zeros(rows, 4, device="cuda")
    x[:, 0] = z
    w = torch.zeros(128, 4, device="cuda")
    w[:, 0] = 1.0
    y = linear_tanh(x, w, torch.zeros(128, device="cuda"))[:, 0].double()
    ref = torch.tanh(z.double())
    rel = ((y - ref).abs() / ref.abs().clamp_min(1e-38)).max()
    assert float(rel) < 1e-6, float(rel)  # <= 8 ulp; the cancelling form gives ~1e-3 at z = 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("k_next,n", [(256, 512), (512, 512), (512, 256), (4, 128), (64, 256), (4, 256), (8, 512),
                                      (8, 384)])
@pytest.mark.parametrize("rows", [1, 127, 129, 4133, 70_000, 65_536])
def test_linear_tanh_backward_gpu(rows, k_next, n):
    """vss_linear_tanh_backward vs fp64: gz = (gz_next @ w_next) * (1 - y^2) and db = gz.sum(0);
    deterministic (the same call twice gives the same bits)."""
    g = torch.Generator(device="cuda").manual_seed(rows * 3 + k_next + n)
    gn = torch.randn(rows, k_next, device="cuda", generator=g) * 1e-3
    wn = torch.randn(k_next, n, device="cuda", generator=g) * (1.0 / k_next) ** 0.5
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g) * 2)
    gz, db = linear_tanh_backward(gn, wn, y)
    ref = (gn.double() @ wn.double()) * (1 - y.double() ** 2)
    scale = float((gn.double().abs() @ wn.double().abs()).max())
    assert float((gz.double() - ref).abs().max()) < 1.2e-7 * k_next * scale + 1e-12  # ~ 2 k u sum|g w|
    torch.testing.assert_close(db.double(), ref.sum(0), rtol=1e-5, atol=1e-6 * scale * (rows ** 0.5 + 1))
    gz2, db2 = linear_tanh_backward(gn, wn, y)
    assert torch.equal(gz, gz2) and torch.equal(db, db2)


def test_output_backward_cpu_formula_matches_autograd():
    """output_backward's CPU form (what the CPU suite's PPO loop runs) against autograd through
    Linear(n -> k_out) over tanh: the hidden pre-activation gradient, its bias and the output dW."""
    g = torch.Generator().manual_seed(5)
    z = torch.randn(33, 128, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(2, 128, generator=g, dtype=torch.float64, requires_grad=True)
    y = torch.tanh(z)
    out = y @ w.t()
    gout = torch.randn(33, 2, generator=g, dtype=torch.float64)
    gz_ref, gw_ref = torch.autograd.grad(out, [z, w], gout)
    gz, db, dw = output_backward(gout, w.detach(), y.detach())
    torch.testing.assert_close(gz, gz_ref)
    torch.testing.assert_close(db, gz_ref.sum(0))
    torch.testing.assert_close(dw, gw_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("k_out,n", [(1, 256), (2, 256), (6, 256), (4, 128), (8, 512), (3, 1024)])
@pytest.mark.parametrize("rows", [1, 3, 127, 4133, 70_000, 65_536])
def test_output_backward_gpu(rows, k_out, n):
    """vss_output_backward vs fp64: gz = (g_out @ w_out) * (1 - y^2), db = gz.sum(0), dw = g_out.T @ y;
    deterministic (the same call twice gives the same bits)."""
    g = torch.Generator(device="cuda").manual_seed(rows * 7 + k_out + n)
    go = torch.randn(rows, k_out, device="cuda", generator=g) * 1e-2
    wo = torch.randn(k_out, n, device="cuda", generator=g) * 0.1
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g) * 2)
    gz, db, dw = output_backward(go, wo, y)
    ref = (go.double() @ wo.double()) * (1 - y.double() ** 2)
    scale = float((go.double().abs() @ wo.double().abs()).max())
    assert float((gz.double() - ref).abs().max()) < 1.2e-7 * 8 * scale + 1e-12
    torch.testing.assert_close(db.double(), ref.sum(0), rtol=1e-5, atol=1e-6 * scale * (rows ** 0.5 + 1))
    dw_ref = go.double().t() @ y.double()
    wscale = float((go.double().abs().t() @ y.double().abs()).max())
    torch.testing.assert_close(dw.double(), dw_ref, rtol=1e-5, atol=2e-7 * wscale * (rows ** 0.5 + 1) + 1e-12)
    gz2, db2, dw2 = output_backward(go, wo, y)
    assert torch.equal(gz, gz2) and torch.equal(db, db2) and torch.equal(dw, dw2)


@pytest.mark.gpu
def test_output_backward_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 16, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_output_backward_chunks(4, 4, 384) == -1  # 1024 % n
    assert lib.vss_output_backward_chunks(4, 6, 256) == -1  # k_pad in {4, 8}
    assert lib.vss_output_backward_chunks(4, 4, 256) > 0
    assert lib.vss_output_backward(s, 4, 4, 256, p, p, p, p, p, None) != 0
    assert lib.vss_output_backward(s, 4, 4, 256, p + 4, p, p, p, p, p) != 0  # misaligned
    with pytest.raises(ValueError):
        output_backward(buf[:36].view(4, 9), buf[:9 * 256].view(9, 256), buf[:1024].view(4, 256))


@pytest.mark.gpu
def test_fused_gemm_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 16, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_linear_tanh(s, 4, 8, 100, p, p, p, p) != 0  # n % 128
    assert lib.vss_linear_tanh(s, 4, 6, 128, p, p, p, p) != 0  # k % 4
    assert lib.vss_linear_tanh(s, 4, 8, 128, p + 4, p, p, p) != 0  # misaligned
    assert lib.vss_linear_tanh_backward(s, 4, 8, 128, p, p, p, p, None) != 0
    assert lib.vss_linear_tanh_backward_chunks(4, 8, 100) == -1
    with pytest.raises(ValueError):
        linear_tanh(buf[:64].view(8, 8), buf[:800].view(100, 8), buf[:100])


@pytest.mark.gpu
@pytest.mark.parametrize("act_dim", [2, 6])
@pytest.mark.parametrize("gemm", ["x6", "fp32"])
@pytest.mark.parametrize("rows", [256, 65536 + 64 * 3])
def test_update_gradients_through_hip_match_autograd_gpu(rows, gemm, act_dim, monkeypatch):
    """The update's forward equals the Agent's within fp32 GEMM rounding (the bf16x6 GEMMs where the
    shapes are exact -- all of them at 256 rows, the weight gradients only at 65,728 -- or the fp32-MFMA
    ones); its gradients (fused HIP GEMM epilogues, split weight gradients) equal autograd's up to fp32
    summation order.  act_dim 6 (the CMA actor: 6 output columns padded to k_pad = 8 in
    vss_output_backward) as well as 2 (SA/DMA: k_pad = 4; the 1-column critic pads to 4 in both)."""
    monkeypatch.setattr(M, "UPDATE_GEMM", gemm)
    agent = make_agent(act_dim).cuda()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(rows, 52, device="cuda", generator=g)
    a = torch.randn(rows, act_dim, device="cuda", generator=g) * 0.5
    outs_ref = agent.get_action_and_value(x, a)
    loss_ref = outs_ref[1].sum() + outs_ref[2].sum() + outs_ref[3].sum()
    grads_ref = torch.autograd.grad(loss_ref, list(agent.parameters()))
    outs = P.get_action_and_value_update(agent, x, a)
    tol = 2e-5
    for u, v in zip(outs[1:], outs_ref[1:]):
        torch.testing.assert_close(u, v, rtol=tol, atol=tol)
    loss = outs[1].sum() + outs[2].sum() + outs[3].sum()
    grads = torch.autograd.grad(loss, list(agent.parameters()))
    for (name, _), u, v in zip(agent.named_parameters(), grads, grads_ref):
        torch.testing.assert_close(u, v, rtol=2e-4, atol=2e-4 * float(v.abs().max()) + 1e-6, msg=name)


@pytest.mark.gpu
@pytest.mark.parametrize("k_out", [1, 2, 6])
@pytest.mark.parametrize("rows", [256, 2048 + 256])
def test_linear_tanh_out_matches_linear_tanh_and_addmm_gpu(rows, k_out):
    """vss_linear_tanh_out (the last hidden layer with the output layer folded into its epilogue,
    ppo…:104-111): y bit-identical to vss_linear_tanh (same kernel body), the output layer within
    fp32 summation-order rounding of addmm."""
    from vss_amd.update import linear_tanh_out
    g = torch.Generator(device="cuda").manual_seed(rows + k_out)
    x = torch.randn(rows, 512, device="cuda", generator=g)
    w = torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(256, device="cuda", generator=g) * 0.1
    w_o = torch.randn(k_out, 256, device="cuda", generator=g) / 16
    b_o = torch.randn(k_out, device="cuda", generator=g)
    y, out = linear_tanh_out(x, w, b, w_o, b_o)
    assert torch.equal(y, linear_tanh(x, w, b))
    want = torch.addmm(b_o.double(), y.double(), w_o.double().t()).float()
    torch.testing.assert_close(out, want, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_linear_tanh_out_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 20, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_linear_tanh_out(s, 200, 512, 256, p, p, p, p, 2, p, p) != 0   # rows % 256
    assert lib.vss_linear_tanh_out(s, 256, 512, 512, p, p, p, p, 2, p, p) != 0   # n_out != 256
    assert lib.vss_linear_tanh_out(s, 256, 512, 256, p, p, p, p, 3, p, p) != 0   # k_out
    assert lib.vss_linear_tanh_out(s, 256, 96, 256, p, p, p, p, 2, p, p) != 0    # k_in % 64
    assert lib.vss_linear_tanh_out(s, 256, 512, 256, p, p, p, p, 2, p + 4, p) != 0  # misaligned w_out


@pytest.mark.gpu
def test_update_gradients_on_rollout_data_at_fp32_error_gpu():
    """The update's gradients on the PPO update's own distributions, not random matrices: observations
    from 64 steps of the fused SA env at 4,096 fields (262,144 rows), actions drawn from the Agent's
    policy, old log-probs within ~0.1 of the current ones (ratios around 1, some clipped), normalised
    advantages.  The default path (x6 GEMMs in fp32 arithmetic + the fused loss) and torch's plain fp32
    autograd (hipBLASLt GEMMs) are both compared with an fp64 evaluation of the same loss: the x6
    path's relative gradient error is at most 1.25 x torch fp32's over the whole gradient and per
    weight matrix (2 x for a matrix whose fp32 error is already below 1e-6), and below 1e-5."""
    from envs.vss import VSS, default_cfg
    from envs.wrappers import SingleAgent
    from vss_amd.loss import ppo_loss, reference_loss
    n, T = 4096, 64
    env = VSS(default_cfg(n), "cuda:0", "cuda:0", 0, True, False, False)
    W = SingleAgent(env)
    g = torch.Generator(device="cuda").manual_seed(11)
    obs = []
    o = W.reset()["obs"]
    for _ in range(T):
        obs.append(o.clone())
        o = W.step(torch.rand((n, 2), device="cuda", generator=g) * 2 - 1)[0]["obs"]
    x = torch.cat(obs)
    rows = x.shape[0]
    agent = make_agent(2).cuda()
    with torch.no_grad():
        act, lp, _, v = agent.get_action_and_value(x)
    logp_old = lp + torch.randn(rows, device="cuda", generator=g) * 0.1
    adv = torch.randn(rows, device="cuda", generator=g)
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ret = v.view(-1) + torch.randn(rows, device="cuda", generator=g) * 0.5
    val = v.view(-1).clone()
    coef = (0.2, 0.005, 4.0, False)
    params = list(agent.parameters())

    def grads(loss_fn, ag, dtype):
        xs = [t.to(dtype) for t in (x, act, logp_old, adv, ret, val)]
        loss, _ = loss_fn(ag, *xs)
        return [t.double() for t in torch.autograd.grad(loss, list(ag.parameters()))]

    def product(ag, x_, a_, lp_, ad_, r_, v_):  # the update's path: _TanhMLP (x6) + vss_ppo_loss
        return ppo_loss(M.mlp_forward(ag.actor_mean, x_), ag.actor_logstd, M.mlp_forward(ag.critic, x_), a_, lp_, ad_,
                        r_, v_, *coef)

    def plain(ag, x_, a_, lp_, ad_, r_, v_):  # torch autograd of the reference's expressions
        return reference_loss(ag.actor_mean(x_), ag.actor_logstd, ag.critic(x_), a_, lp_, ad_, r_, v_, *coef)

    g6 = grads(product, agent, torch.float32)
    gt = grads(plain, agent, torch.float32)
    import copy
    g64 = grads(plain, copy.deepcopy(agent).double(), torch.float64)
    flat = lambda gs: torch.cat([t.reshape(-1) for t in gs])  # noqa: E731
    e6 = float((flat(g6) - flat(g64)).norm() / flat(g64).norm())
    et = float((flat(gt) - flat(g64)).norm() / flat(g64).norm())
    assert e6 <= 1.25 * et and e6 < 1e-5, (e6, et)
    for (name, p), a, b, c in zip(agent.named_parameters(), g6, gt, g64):
        if p.dim() != 2:
            continue
        ea = float((a - c).norm() / c.norm())
        eb = float((b - c).norm() / c.norm())
        assert ea <= (1.25 if eb >= 1e-6 else 2.0) * eb + 1e-9 and ea < 1e-5, (name, ea, eb)
