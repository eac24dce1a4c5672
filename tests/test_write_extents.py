"""Write extents of the PPO update's HIP entry points (round-3 VERDICT: rule out an out-of-bounds write by
one of the update kernels, which under a captured graph could land on kernel-argument memory).

Every buffer an entry point is handed -- inputs, outputs, weight-plane scratch, partial-sum parts -- is
a window inside a larger allocation whose 256 KiB on each side hold a NaN bit pattern no kernel writes.
After the call (and a device synchronise) the test asserts, on the host:
  * the guard regions on both sides of every buffer are untouched;
  * every input buffer is bit-identical to its copy from before the call;
  * every output the contract says is written in full (activations, gradients, weight planes, parts)
    holds no sentinel word any more (it was covered, so its caller-side sums read no stale memory).
Shapes: the Agent's layers (ppo_continuous_action_isaacgym.py:135-143: n_in -> 256 -> 512 -> 512 ->
256 -> n_out) at config 3's update minibatch (65,536 envs x 128 / 4 = 2,097,152 rows) and at the
4,095-env minibatch padded to whole tiles (131,072 rows); the loss at both, with and without padding
rows.  The reference's update that these kernels implement: ppo_continuous_action_isaacgym.py:314-357."""
import ctypes

import pytest
import torch

GUARD = 1 << 16  # int32 words on each side (256 KiB)
SENTINEL = 0x7FA5A5A5  # a quiet-NaN bit pattern


class Guarded:
    """A buffer of `shape` and `dtype` inside an int32 allocation with GUARD sentinel words on each side."""

    def __init__(self, shape, dtype=torch.float32, fill=None, dev="cuda"):
        n = 1
        for s in shape:
            n *= s
        elem = torch.empty((), dtype=dtype).element_size()
        self.words = (n * elem + 3) // 4
        self.backing = torch.full((2 * GUARD + self.words,), SENTINEL, dtype=torch.int32, device=dev)
        self.t = self.backing[GUARD:GUARD + self.words].view(dtype)[:n].view(shape)
        if fill is not None:
            self.t.copy_(fill)
        self.before = None

    @property
    def ptr(self):
        return self.t.data_ptr()

    def snapshot(self):
        self.before = self.backing.clone()

    def guards_intact(self):
        b = self.backing
        return bool((b[:GUARD] == SENTINEL).all()) and bool((b[GUARD + self.words:] == SENTINEL).all())

    def unchanged(self):
        return torch.equal(self.backing, self.before)

    def covered(self):
        """No sentinel word left inside the window (every word was written)."""
        return not bool((self.backing[GUARD:GUARD + self.words] == SENTINEL).any())


def _run(name, call, inputs, outputs, full_outputs):
    for g in inputs:
        g.snapshot()
    rc = call()
    torch.cuda.synchronize()
    assert rc == 0, f"{name}: rc {rc}"
    for i, g in enumerate(inputs):
        assert g.guards_intact() and g.unchanged(), f"{name}: input {i} or its guards were written"
    for i, g in enumerate(outputs):
        assert g.guards_intact(), f"{name}: output {i} written outside its extent"
    for i, g in enumerate(full_outputs):
        assert g.covered(), f"{name}: output {i} not written in full"


def _rand(shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(shape, device="cuda", generator=g) * scale


ROWS = [2_097_152, 131_072]


@pytest.fixture(scope="module")
def lib():
    from vss_amd import _native as N
    return N.load()


def _stream():
    from vss_amd import _native as N
    return N.stream_of(torch.device("cuda"))


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ROWS)
def test_forward_entries_write_only_their_outputs_gpu(lib, rows):
    st = _stream()
    # first layer (fp32 small-k kernel): n_in 52 -> 256
    x = Guarded((rows, 52), fill=_rand((rows, 52), 1.0, 1))
    w = Guarded((256, 52), fill=_rand((256, 52), 0.1, 2))
    b = Guarded((256,), fill=_rand((256,), 0.1, 3))
    y = Guarded((rows, 256))
    _run("vss_linear_tanh", lambda: lib.vss_linear_tanh(st, rows, 52, 256, x.ptr, w.ptr, b.ptr, y.ptr),
         [x, w, b], [y], [y])
    del x
    h = y
    # hidden layers on x6: 256 -> 512, 512 -> 512
    for k, n, s in ((256, 512, 4), (512, 512, 7)):
        w = Guarded((n, k), fill=_rand((n, k), 0.05, s))
        b = Guarded((n,), fill=_rand((n,), 0.1, s + 1))
        planes = Guarded((3, n * k), dtype=torch.int16)
        out = Guarded((rows, n))
        _run(f"vss_linear_tanh_bf16x6 {k}->{n}",
             lambda: lib.vss_linear_tanh_bf16x6(st, rows, k, n, h.ptr, w.ptr, b.ptr, out.ptr, planes.ptr),
             [h, w, b], [out, planes], [out, planes])
        h = out
    # the last hidden layer with the output layer folded in: 512 -> 256 -> k_out
    for k_out in (1, 2, 6):
        w = Guarded((256, 512), fill=_rand((256, 512), 0.05, 10))
        b = Guarded((256,), fill=_rand((256,), 0.1, 11))
        wo = Guarded((k_out, 256), fill=_rand((k_out, 256), 0.05, 12))
        planes = Guarded((3, 256 * 512), dtype=torch.int16)
        y = Guarded((rows, 256))
        part = Guarded((4, rows, k_out))
        _run(f"vss_linear_tanh_out_bf16x6 k_out={k_out}",
             lambda: lib.vss_linear_tanh_out_bf16x6(st, rows, 512, 256, h.ptr, w.ptr, b.ptr, y.ptr, k_out, wo.ptr,
                                                    part.ptr, planes.ptr),
             [h, w, b, wo], [y, part, planes], [y, part, planes])


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ROWS)
def test_backward_entries_write_only_their_outputs_gpu(lib, rows):
    st = _stream()
    # the output layer's backward into the 256-wide tanh layer below it (k_pad 4: SA/DMA, 8: CMA)
    y256 = Guarded((rows, 256), fill=torch.tanh(_rand((rows, 256), 1.0, 20)))
    for k_pad in (4, 8):
        g_out = Guarded((rows, k_pad), fill=_rand((rows, k_pad), 0.01, 21))
        w_t = Guarded((256, k_pad), fill=_rand((256, k_pad), 0.05, 22))
        chunks = lib.vss_output_backward_chunks(rows, k_pad, 256)
        assert chunks > 0
        gz = Guarded((rows, 256))
        bpart = Guarded((chunks, 256))
        wpart = Guarded((chunks, k_pad, 256))
        _run(f"vss_output_backward k_pad={k_pad}",
             lambda: lib.vss_output_backward(st, rows, k_pad, 256, g_out.ptr, w_t.ptr, y256.ptr, gz.ptr, bpart.ptr,
                                             wpart.ptr),
             [g_out, w_t, y256], [gz, bpart, wpart], [gz, bpart, wpart])
    # the hidden layers' input gradients through the tanh below (k_next, n): 256 <- 512 <- 512 <- 256
    g_next = Guarded((rows, 256), fill=_rand((rows, 256), 0.01, 23))
    for k_next, n, s in ((256, 512, 30), (512, 512, 33), (512, 256, 36)):
        if g_next.t.shape[1] != k_next:
            g_next = Guarded((rows, k_next), fill=_rand((rows, k_next), 0.01, s))
        w_t = Guarded((n, k_next), fill=_rand((n, k_next), 0.05, s + 1))
        y = Guarded((rows, n), fill=torch.tanh(_rand((rows, n), 1.0, s + 2)))
        chunks = lib.vss_linear_tanh_backward_chunks_bf16x6(rows, k_next, n)
        assert chunks > 0
        gz = Guarded((rows, n))
        part = Guarded((chunks, n))
        planes = Guarded((3, n * k_next), dtype=torch.int16)
        _run(f"vss_linear_tanh_backward_bf16x6 {n}<-{k_next}",
             lambda: lib.vss_linear_tanh_backward_bf16x6(st, rows, k_next, n, g_next.ptr, w_t.ptr, y.ptr, gz.ptr,
                                                         part.ptr, planes.ptr),
             [g_next, w_t, y], [gz, part, planes], [gz, part, planes])
        g_next = gz
        del y
    # the weight gradients (n_out, k_in) of the 256->512, 512->512 and 512->256 layers
    for n_out, k_in, s in ((512, 256, 40), (512, 512, 42), (256, 512, 44)):
        grad = Guarded((rows, n_out), fill=_rand((rows, n_out), 0.01, s))
        x = Guarded((rows, k_in), fill=_rand((rows, k_in), 1.0, s + 1))
        chunks = lib.vss_weight_grad_chunks_bf16x6(rows, n_out, k_in)
        assert chunks > 0
        parts = Guarded((chunks, n_out, k_in))
        _run(f"vss_weight_grad_bf16x6 {n_out}x{k_in}",
             lambda: lib.vss_weight_grad_bf16x6(st, rows, n_out, k_in, grad.ptr, x.ptr, parts.ptr),
             [grad, x], [parts], [parts])
        del grad, x, parts


@pytest.mark.gpu
@pytest.mark.parametrize("rows,rows_pad", [(2_097_152, 2_097_152), (131_040, 131_072), (1000, 1024)])
@pytest.mark.parametrize("n_act", [2, 6])
def test_loss_writes_only_its_outputs_gpu(lib, rows, rows_pad, n_act):
    st = _stream()
    mean = Guarded((rows_pad, n_act), fill=_rand((rows_pad, n_act), 0.5, 50))
    logstd = Guarded((n_act,), fill=_rand((n_act,), 0.3, 51))
    value = Guarded((rows_pad,), fill=_rand((rows_pad,), 1.0, 52))
    action = Guarded((rows_pad, n_act), fill=_rand((rows_pad, n_act), 1.0, 53))
    lp_old = Guarded((rows,), fill=_rand((rows,), 1.0, 54) - 2.0)
    adv = Guarded((rows,), fill=_rand((rows,), 1.0, 55))
    ret = Guarded((rows,), fill=_rand((rows,), 1.0, 56))
    v_old = Guarded((rows,), fill=_rand((rows,), 1.0, 57))
    scratch = lib.vss_ppo_loss_scratch_floats(rows_pad, n_act)
    assert scratch > 0
    g_mean = Guarded((rows_pad, n_act))
    g_value = Guarded((rows_pad,))
    g_logstd = Guarded((n_act,))
    loss = Guarded((1,))
    stats = Guarded((6,))
    partial = Guarded((scratch,))
    f = ctypes.c_float
    for clip_vloss in (0, 1):
        _run(f"vss_ppo_loss clip_vloss={clip_vloss}",
             lambda: lib.vss_ppo_loss(st, rows, rows_pad, n_act, mean.ptr, logstd.ptr, value.ptr, action.ptr,
                                      lp_old.ptr, adv.ptr, ret.ptr, v_old.ptr, f(0.2), f(0.8), f(1.2), f(0.005),
                                      f(4.0), clip_vloss, g_mean.ptr, g_value.ptr, g_logstd.ptr, loss.ptr, stats.ptr,
                                      partial.ptr),
             [mean, logstd, value, action, lp_old, adv, ret, v_old],
             [g_mean, g_value, g_logstd, loss, stats, partial], [g_mean, g_value, g_logstd, loss, stats])
