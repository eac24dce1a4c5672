"""PPO-update helper vss_tanh_grad_bias (csrc/vss_update.hip): one HIP pass for the backward of a
hidden tanh layer, checked against torch's tanh_backward + bias-gradient reduction (the fp32
reference of the same op), and the update's gradients through it against plain autograd."""
import pytest
import torch

import ppo_continuous_action_isaacgym as P
from vss_amd import _native as N
from vss_amd.update import tanh_grad_bias

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


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [256, 65536 + 64 * 3])
def test_update_gradients_through_hip_match_autograd_gpu(rows):
    """The update's forward (addmm + in-place tanh) equals the Agent's; its gradients (HIP tanh
    backward + bias, split-K dW) equal autograd's up to fp32 summation order."""
    agent = make_agent(2).cuda()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(rows, 52, device="cuda", generator=g)
    a = torch.randn(rows, 2, device="cuda", generator=g) * 0.5
    outs_ref = agent.get_action_and_value(x, a)
    loss_ref = outs_ref[1].sum() + outs_ref[2].sum() + outs_ref[3].sum()
    grads_ref = torch.autograd.grad(loss_ref, list(agent.parameters()))
    outs = P.get_action_and_value_update(agent, x, a)
    for u, v in zip(outs[1:], outs_ref[1:]):
        torch.testing.assert_close(u, v, rtol=0, atol=0)
    loss = outs[1].sum() + outs[2].sum() + outs[3].sum()
    grads = torch.autograd.grad(loss, list(agent.parameters()))
    for (name, _), u, v in zip(agent.named_parameters(), grads, grads_ref):
        torch.testing.assert_close(u, v, rtol=2e-4, atol=2e-4 * float(v.abs().max()) + 1e-6, msg=name)
