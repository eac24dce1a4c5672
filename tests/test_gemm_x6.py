"""The update's GEMMs in fp32 arithmetic on the bf16 matrix cores (csrc/vss_gemm_x6.hip): every fp32
operand split exactly into three bf16 parts, the six partial products above 2^-23 |a||b| summed in
fp32.  Checked against fp64 evaluations of the same functions, beside the fp32 GEMMs they replace
(hipBLASLt's torch.mm / addmm and the fp32-MFMA kernels of csrc/vss_update.hip): the bar is the
fp32 GEMM's own error (tolerance in each test), plus exact results where fp32 is exact (integer
operands) and the per-product bound of the split (one-row outer products)."""
import pytest
import torch

from vss_amd import _native as N
from vss_amd.update import (first_layer_x6, first_layer_x6_ok, first_weight_grad_x6, first_wgrad_ok, linear_tanh,
                            linear_tanh_backward,
                            linear_tanh_backward_mixed, linear_tanh_backward_x6,
                            linear_tanh_mixed, linear_tanh_out_mixed, linear_tanh_out_x6, linear_tanh_x6,
                            weight_grad_mixed, weight_grad_x6, x6_ok, x6_wgrad_ok)


def test_x6_shape_predicates_cpu():
    assert x6_ok(2097152, 512, 256) and x6_ok(256, 256, 512) and x6_ok(256, 64, 128)
    assert not x6_ok(200, 512, 256) and not x6_ok(256, 52, 256) and not x6_ok(256, 512, 100)
    assert x6_wgrad_ok(64, 256, 128) and x6_wgrad_ok(2097152, 512, 512)
    assert not x6_wgrad_ok(100, 256, 128) and not x6_wgrad_ok(64, 128, 128) and not x6_wgrad_ok(64, 256, 52)


def test_first_wgrad_shape_predicate_cpu():
    """The first layer's weight gradient (nn.Linear(52, 256)): n_out 256, k_in <= 64 and % 4, rows % 64."""
    assert first_wgrad_ok(2097152, 256, 52) and first_wgrad_ok(64, 256, 64) and first_wgrad_ok(131008, 256, 4)
    assert not first_wgrad_ok(100, 256, 52) and not first_wgrad_ok(64, 512, 52) and not first_wgrad_ok(64, 256, 68)
    assert not first_wgrad_ok(64, 256, 50)
    with pytest.raises(ValueError):
        first_weight_grad_x6(torch.zeros(64, 256), torch.zeros(64, 52))


def test_x6_refuses_cpu_tensors():
    x = torch.zeros(256, 64)
    with pytest.raises(ValueError):
        linear_tanh_x6(x, torch.zeros(128, 64), torch.zeros(128))
    with pytest.raises(ValueError):
        weight_grad_x6(torch.zeros(64, 256), torch.zeros(64, 128))


def _rel(out, ref64):
    d = out.double() - ref64
    return float(d.abs().max() / ref64.abs().max()), float(d.norm() / ref64.norm())


def _ops(rows, k, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    gz = torch.randn(rows, n, device="cuda", generator=g) * 1e-3
    y_lo = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    return x, w, b, gz, y_lo


SHAPES = [(256, 512), (512, 512), (512, 256), (64, 128), (128, 256)]   # (k, n) forward
BSHAPES = [(256, 512), (512, 512), (512, 256), (128, 256), (256, 128)]  # backward: from n into k


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", SHAPES)
@pytest.mark.parametrize("rows", [256, 8192])
def test_x6_forward_error_at_most_fp32_gpu(rows, k, n):
    """y = tanh(x W^T + b): error vs fp64 no larger than hipBLASLt's fp32 addmm + tanh (x 1.25 slack)
    and below 4e-6 of max|y| (tolerance)."""
    x, w, b, _, _ = _ops(rows, k, n, rows + k * n)
    ref = torch.tanh(x.double() @ w.double().t() + b.double())
    e6 = _rel(linear_tanh_x6(x, w, b), ref)
    et = _rel(torch.addmm(b, x, w.t()).tanh_(), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * et[1] + 1e-8, (e6, et)


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", BSHAPES)
@pytest.mark.parametrize("rows", [256, 8192])
def test_x6_backward_error_at_most_fp32_gpu(rows, k, n):
    """gz = (g W) * (1 - y^2) and its column sums (the bias gradient): error vs fp64 no larger than
    torch's fp32 mm (x 1.25 slack); the column sums within 1e-5 relative."""
    x, w, _, gz, y_lo = _ops(rows, k, n, 3 * rows + k + n)
    ref = (gz.double() @ w.double()) * (1 - y_lo.double() ** 2)
    g6, db6 = linear_tanh_backward_x6(gz, w, y_lo)
    e6 = _rel(g6, ref)
    et = _rel(gz.mm(w) * (1 - y_lo * y_lo), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * et[1] + 1e-8, (e6, et)
    torch.testing.assert_close(db6.double(), ref.sum(0), rtol=1e-5, atol=1e-5 * float(ref.sum(0).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("n_out,k_in", [(512, 512), (512, 256), (256, 512), (256, 128)])
@pytest.mark.parametrize("rows", [64, 8192, 65536 + 64])
def test_x6_weight_grad_error_at_most_fp32_gpu(rows, n_out, k_in):
    """dW = g^T x over the rows (split in parts): error vs fp64 no larger than torch's fp32 mm."""
    g = torch.Generator(device="cuda").manual_seed(rows + n_out + k_in)
    gz = torch.randn(rows, n_out, device="cuda", generator=g) * 1e-3
    x = torch.tanh(torch.randn(rows, k_in, device="cuda", generator=g))
    ref = gz.double().t() @ x.double()
    e6 = _rel(weight_grad_x6(gz, x), ref)
    et = _rel(gz.t().mm(x), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * et[1] + 1e-8, (e6, et)


@pytest.mark.gpu
@pytest.mark.parametrize("k_in", [52, 4, 64, 36])
@pytest.mark.parametrize("rows", [64, 8192, 131008, 2097152])
def test_x6_first_layer_weight_grad_error_at_most_fp32_gpu(rows, k_in):
    """The first layer's dW = g^T x (g (rows, 256), x (rows, k_in): the observations, 52 wide in the
    Agent) on vss_first_weight_grad_bf16x6: error vs fp64 no larger than torch's fp32 mm (x 1.25), and
    two calls give the same bits (fixed-order parts)."""
    g = torch.Generator(device="cuda").manual_seed(rows + k_in)
    gz = torch.randn(rows, 256, device="cuda", generator=g) * 1e-3
    x = torch.randn(rows, k_in, device="cuda", generator=g) * 2.0
    ref = gz.double().t() @ x.double()
    got = first_weight_grad_x6(gz, x)
    assert got.shape == (256, k_in)
    e6 = _rel(got, ref)
    et = _rel(gz.t().mm(x), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * et[1] + 1e-8, (e6, et)
    assert torch.equal(got, first_weight_grad_x6(gz, x))


@pytest.mark.gpu
def test_x6_first_layer_weight_grad_exact_and_per_product_gpu():
    """Integer operands with exact fp32 sums give the exact dW; one nonzero row (an outer product of
    full 24-bit values) is within 2^-22 |a b| of each product; a strided minibatch view (rows of a
    larger observation buffer) gives the contiguous copy's bits."""
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = 4096
    gi = torch.randint(-100, 101, (rows, 256), device="cuda", generator=g).float()
    xi = torch.randint(-300, 301, (rows, 52), device="cuda", generator=g).float()
    assert torch.equal(first_weight_grad_x6(gi, xi).double(), gi.double().t() @ xi.double())
    gz = torch.zeros(128, 256, device="cuda")
    x = torch.zeros(128, 52, device="cuda")
    gz[77] = torch.randn(256, device="cuda", generator=g) * 3.7
    x[77] = torch.randn(52, device="cuda", generator=g) * 0.31
    ref = gz[77].double()[:, None] * x[77].double()[None, :]
    rel = ((first_weight_grad_x6(gz, x).double() - ref).abs() / ref.abs().clamp_min(1e-300)).max()
    assert float(rel) <= 2 ** -22, float(rel)
    big = torch.randn(2 * rows, 52, device="cuda", generator=g)
    gz = torch.randn(rows, 256, device="cuda", generator=g)
    assert torch.equal(first_weight_grad_x6(gz, big[::2]), first_weight_grad_x6(gz, big[::2].contiguous()))


def test_first_layer_x6_shape_predicate_cpu():
    """The first layer's forward (nn.Linear(52, 256) + Tanh): n 256, k <= 64 and % 4, any rows."""
    assert first_layer_x6_ok(52, 256) and first_layer_x6_ok(4, 256) and first_layer_x6_ok(64, 256)
    assert not first_layer_x6_ok(68, 256) and not first_layer_x6_ok(50, 256) and not first_layer_x6_ok(52, 512)
    with pytest.raises(ValueError):
        first_layer_x6(torch.zeros(16, 52), torch.zeros(256, 52), torch.zeros(256))


@pytest.mark.gpu
@pytest.mark.parametrize("k_in", [52, 4, 64, 36])
@pytest.mark.parametrize("rows", [1, 17, 4096 + 5, 131040, 2097152])
def test_x6_first_layer_forward_error_at_most_fp32_gpu(rows, k_in):
    """The first layer's y = tanh(x W^T + b) on vss_first_layer_bf16x6 (x the observations, any row
    count): error vs fp64 no larger than the fp32-MFMA first_layer_kernel's (vss_linear_tanh, the
    kernel it replaces, with the same tanh_f32; x 1.25 slack), below 4e-6 of max|y|; two calls give the
    same bits.  (hipBLASLt's addmm + torch's tanh is printed beside: at small k its error is torch's
    correctly rounded tanh, not the GEMM.)"""
    g = torch.Generator(device="cuda").manual_seed(rows + k_in)
    x = torch.randn(rows, k_in, device="cuda", generator=g) * 1.5
    w = torch.randn(256, k_in, device="cuda", generator=g) * (2.0 / k_in) ** 0.5
    b = torch.randn(256, device="cuda", generator=g) * 0.1
    n = min(rows, 65536)
    ref = torch.tanh(x[:n].double() @ w.double().t() + b.double())
    got = first_layer_x6(x, w, b)
    assert got.shape == (rows, 256)
    e6 = _rel(got[:n], ref)
    ef = _rel(linear_tanh(x, w, b)[:n], ref)
    et = _rel(torch.addmm(b, x[:n], w.t()).tanh_(), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * ef[1] + 1e-8, (e6, ef, et)
    assert torch.equal(got, first_layer_x6(x, w, b))


@pytest.mark.gpu
def test_x6_first_layer_forward_exact_and_in_the_update_gpu():
    """Integer operands with exact fp32 sums: the same bits as the fp32-MFMA kernel (both take tanh_f32
    of the exact pre-activation); a strided minibatch view gives the contiguous copy's bits; and
    linear_tanh_mixed (the update's and the rollout chain's first layer) runs this kernel."""
    g = torch.Generator(device="cuda").manual_seed(5)
    rows = 4096 + 3
    xi = torch.randint(-3, 4, (rows, 52), device="cuda", generator=g).float()
    wi = torch.randint(-2, 3, (256, 52), device="cuda", generator=g).float() / 64
    bi = torch.randint(-8, 9, (256,), device="cuda", generator=g).float() / 16
    assert torch.equal(first_layer_x6(xi, wi, bi), linear_tanh(xi, wi, bi))
    big = torch.randn(2 * rows, 52, device="cuda", generator=g)
    w = torch.randn(256, 52, device="cuda", generator=g) * 0.2
    b = torch.randn(256, device="cuda", generator=g) * 0.1
    assert torch.equal(first_layer_x6(big[::2], w, b), first_layer_x6(big[::2].contiguous(), w, b))
    assert torch.equal(linear_tanh_mixed(big[:rows], w, b), first_layer_x6(big[:rows], w, b))


@pytest.mark.gpu
def test_x6_first_layer_forward_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 20, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_first_layer_bf16x6(s, 64, 68, 256, p, p, p, p) != 0  # k_in > 64
    assert lib.vss_first_layer_bf16x6(s, 64, 50, 256, p, p, p, p) != 0  # k_in % 4
    assert lib.vss_first_layer_bf16x6(s, 64, 52, 512, p, p, p, p) != 0  # n_out != 256
    assert lib.vss_first_layer_bf16x6(s, 64, 52, 256, p + 4, p, p, p) != 0  # misaligned x
    assert lib.vss_first_layer_bf16x6(s, 64, 52, 256, p, p, p, p + 4) != 0  # misaligned y
    assert lib.vss_first_layer_bf16x6(s, 0, 52, 256, p, p, p, p) == 0


@pytest.mark.gpu
def test_x6_first_layer_weight_grad_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 20, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_first_weight_grad_chunks_bf16x6(100, 256, 52) == -1  # rows % 64
    assert lib.vss_first_weight_grad_chunks_bf16x6(64, 512, 52) == -1   # n_out != 256
    assert lib.vss_first_weight_grad_chunks_bf16x6(64, 256, 68) == -1   # k_in > 64
    assert lib.vss_first_weight_grad_chunks_bf16x6(64, 256, 50) == -1   # k_in % 4
    assert lib.vss_first_weight_grad_chunks_bf16x6(2097152, 256, 52) == 256
    assert lib.vss_first_weight_grad_bf16x6(s, 64, 256, 52, p + 4, p, p) != 0  # misaligned grad
    assert lib.vss_first_weight_grad_bf16x6(s, 64, 256, 52, p, p, None) != 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [128, 384])
def test_x6_persistent_multi_item_cfga_gpu(n):
    """Widths that are not multiples of 256 take the 128-feature x 256-row block (CfgA); at 131,072 rows
    every block runs several work items (n = 128: 512 items on 256 blocks; n = 384: 1,536 items on
    240 blocks with a fixed i tile per block), so the bias and column-sum bookkeeping of one i tile
    per block is exercised across items.  Forward, backward and the column sums vs fp64."""
    rows, k = 131072, 256
    x, w, b, _, _ = _ops(rows, k, n, n)
    ref = torch.tanh(x.double() @ w.double().t() + b.double())
    e6 = _rel(linear_tanh_x6(x, w, b), ref)
    assert e6[0] < 4e-6, e6
    # backward from this n-wide layer into a k-wide tanh layer: P = W^T (k, n) -> n_out = k = 256 (CfgB)
    # and from a k-wide layer into the n-wide one: n_out = n (CfgA, multi-item)
    g = torch.Generator(device="cuda").manual_seed(n + 1)
    w2 = torch.randn(k, n, device="cuda", generator=g) / k ** 0.5
    g_next = torch.randn(rows, k, device="cuda", generator=g) * 1e-3
    y_n = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    refb = (g_next.double() @ w2.double()) * (1 - y_n.double() ** 2)
    gz, db = linear_tanh_backward_x6(g_next, w2, y_n)
    eb = _rel(gz, refb)
    et = _rel(g_next.mm(w2) * (1 - y_n * y_n), refb)
    assert eb[0] < 4e-6 and eb[1] < 1.25 * et[1] + 1e-8, (eb, et)
    torch.testing.assert_close(db.double(), refb.sum(0), rtol=1e-5, atol=1e-5 * float(refb.sum(0).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("n_out,k_in", [(256, 384), (512, 384)])
def test_x6_weight_grad_k_in_384_gpu(n_out, k_in):
    """k_in = 384 (3 i tiles): the grid trim (grid -= grid % 8) leaves some blocks two work items;
    the result against fp64 at the fp32 GEMM's error."""
    rows = 65536 + 64
    g = torch.Generator(device="cuda").manual_seed(n_out + k_in)
    gz = torch.randn(rows, n_out, device="cuda", generator=g) * 1e-3
    x = torch.tanh(torch.randn(rows, k_in, device="cuda", generator=g))
    ref = gz.double().t() @ x.double()
    e6 = _rel(weight_grad_x6(gz, x), ref)
    et = _rel(gz.t().mm(x), ref)
    assert e6[0] < 4e-6 and e6[1] < 1.25 * et[1] + 1e-8, (e6, et)


@pytest.mark.gpu
def test_x6_exact_on_integer_operands_gpu():
    """Integer operands with exact fp32 sums: every entry point returns the exact result (the split of
    an integer of <= 24 bits is exact, the six products carry all of it for <= 16-bit factors)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    rows, k, n = 512, 128, 256
    x = torch.randint(-300, 301, (rows, k), device="cuda", generator=g).float()
    w = torch.randint(-200, 201, (n, k), device="cuda", generator=g).float()
    exact = x.double() @ w.double().t()
    assert float(exact.abs().max()) < 2 ** 24
    # weight gradient: grad (rows, n) integer, x (rows, k) integer
    gi = torch.randint(-100, 101, (rows, n), device="cuda", generator=g).float()
    wg = weight_grad_x6(gi, x)
    assert torch.equal(wg.double(), gi.double().t() @ x.double())
    # backward with y = 0 (1 - y^2 = 1): gz = g W exactly; the column sums are exact too
    gz, db = linear_tanh_backward_x6(gi, w, torch.zeros(rows, k, device="cuda"))
    want = gi.double() @ w.double()
    assert torch.equal(gz.double(), want)
    assert torch.equal(db.double(), want.sum(0))


@pytest.mark.gpu
def test_x6_split_bound_per_product_gpu():
    """One row (an outer product): each output is ONE product a b of full 24-bit fp32 values; the split
    keeps it within 2^-22 |a b| (the dropped partial products are below 2^-23 |a b|, plus the fp32
    rounding of the sum)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    gz = torch.zeros(64, 256, device="cuda")
    x = torch.zeros(64, 128, device="cuda")
    gz[17] = torch.randn(256, device="cuda", generator=g) * 3.7
    x[17] = torch.randn(128, device="cuda", generator=g) * 0.31
    ref = gz[17].double()[:, None] * x[17].double()[None, :]
    rel = ((weight_grad_x6(gz, x).double() - ref).abs() / ref.abs().clamp_min(1e-300)).max()
    assert float(rel) <= 2 ** -22, float(rel)


@pytest.mark.gpu
@pytest.mark.parametrize("k_out", [1, 2, 6])
def test_x6_linear_tanh_out_gpu(k_out):
    """The last hidden layer with the output layer folded in: y as linear_tanh_x6 (same kernel body,
    bit for bit), the output within fp32 rounding of an fp64 evaluation on that y."""
    g = torch.Generator(device="cuda").manual_seed(k_out)
    rows = 2048 + 256
    x = torch.randn(rows, 512, device="cuda", generator=g)
    w = torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(256, device="cuda", generator=g) * 0.1
    w_o = torch.randn(k_out, 256, device="cuda", generator=g) / 16
    b_o = torch.randn(k_out, device="cuda", generator=g)
    y, out = linear_tanh_out_x6(x, w, b, w_o, b_o)
    assert torch.equal(y, linear_tanh_x6(x, w, b))
    want = torch.addmm(b_o.double(), y.double(), w_o.double().t()).float()
    torch.testing.assert_close(out, want, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_x6_matches_fp32_mfma_kernels_gpu():
    """The bf16x6 and fp32-MFMA kernels compute the same functions: equal within fp32 rounding."""
    x, w, b, gz, y_lo = _ops(4096, 512, 256, 9)
    torch.testing.assert_close(linear_tanh_x6(x, w, b), linear_tanh(x, w, b), rtol=1e-5, atol=2e-6)
    g6, d6 = linear_tanh_backward_x6(gz, w, y_lo)
    gf, df = linear_tanh_backward(gz, w, y_lo)
    torch.testing.assert_close(g6, gf, rtol=1e-5, atol=1e-5 * float(gf.abs().max()))
    torch.testing.assert_close(d6, df, rtol=1e-5, atol=1e-5 * float(df.abs().max()))


@pytest.mark.gpu
def test_x6_refusals_gpu():
    lib = N.load()
    buf = torch.zeros(1 << 20, device="cuda")
    p, s = buf.data_ptr(), N.stream_of(buf.device)
    assert lib.vss_linear_tanh_bf16x6(s, 200, 512, 256, p, p, p, p, p) != 0      # rows % 256
    assert lib.vss_linear_tanh_bf16x6(s, 256, 96, 256, p, p, p, p, p) != 0       # k % 64
    assert lib.vss_linear_tanh_bf16x6(s, 256, 512, 200, p, p, p, p, p) != 0      # n % 128
    assert lib.vss_linear_tanh_bf16x6(s, 256, 512, 256, p + 4, p, p, p, p) != 0  # misaligned
    assert lib.vss_linear_tanh_bf16x6(s, 256, 512, 256, p, p, p, p, None) != 0  # no scratch
    assert lib.vss_linear_tanh_out_bf16x6(s, 256, 512, 512, p, p, p, p, 2, p, p, p) != 0  # n_out != 256
    assert lib.vss_linear_tanh_out_bf16x6(s, 256, 512, 256, p, p, p, p, 3, p, p, p) != 0  # k_out
    assert lib.vss_linear_tanh_backward_bf16x6(s, 256, 512, 256, p, p, p, p, None, p) != 0
    assert lib.vss_linear_tanh_backward_chunks_bf16x6(200, 512, 256) == -1
    assert lib.vss_weight_grad_chunks_bf16x6(100, 256, 128) == -1
    assert lib.vss_weight_grad_chunks_bf16x6(64, 128, 128) == -1
    assert lib.vss_weight_grad_bf16x6(s, 64, 256, 52, p, p, p) != 0
    assert lib.vss_weight_grad_bf16x6(s, 64, 256, 128, p, p, None) != 0


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [100, 256, 300, 131040])
def test_mixed_rows_match_fp64_gpu(rows):
    """Row counts that are not tile multiples (the reference's default minibatch: 4,095 envs x 128 / 4
    = 131,040 rows): the whole tiles on the x6 kernels, the ragged rest on hipBLASLt (below one tile:
    the fp32-MFMA kernels), one result within the fp32 tolerances of the single-kernel tests."""
    x, w, b, gz, y_lo = _ops(rows, 512, 256, rows)
    ref = torch.tanh(x.double() @ w.double().t() + b.double())
    y = linear_tanh_mixed(x, w, b)
    assert _rel(y, ref)[0] < 4e-6
    main = rows // 256 * 256
    if 0 < main < rows:  # the ragged tail: hipBLASLt addmm + tanh, as torch computes it
        torch.testing.assert_close(y[main:], torch.addmm(b, x[main:], w.t()).tanh_(), rtol=0, atol=0)
    wo = torch.randn(6, 256, device="cuda") / 16
    bo = torch.randn(6, device="cuda") * 0.1
    y2, o2 = linear_tanh_out_mixed(x, w, b, wo, bo)
    assert torch.equal(y2, y)
    torch.testing.assert_close(o2.double(), y.double() @ wo.double().t() + bo.double(), rtol=1e-5, atol=1e-5)
    # backward from the 256-wide layer into a 512-wide tanh layer
    w2 = torch.randn(256, 512, device="cuda") / 16
    y512 = torch.tanh(torch.randn(rows, 512, device="cuda"))
    g256 = torch.randn(rows, 256, device="cuda") * 1e-3
    refb = (g256.double() @ w2.double()) * (1 - y512.double() ** 2)
    gzm, dbm = linear_tanh_backward_mixed(g256, w2, y512)
    assert _rel(gzm, refb)[0] < 4e-6
    torch.testing.assert_close(dbm.double(), refb.sum(0), rtol=1e-5, atol=1e-5 * float(refb.sum(0).abs().max()))
    refw = g256.double().t() @ x.double()
    assert _rel(weight_grad_mixed(g256, x), refw)[0] < 4e-6


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(512, 256), (512, 512), (256, 512), (384, 128)])
def test_weight_planes_feed_the_gemms_bit_exact_gpu(n, k):
    """vss_weight_planes_bf16x6 (several weights' planes in one launch, the backward's W^T read straight
    from the (k_next, n) weight): the GEMM entries given those planes and a NULL weight produce the same
    bits as when they split (and, for the backward, transpose) the weight themselves."""
    from vss_amd.update import linear_tanh_out_x6, weight_planes
    g = torch.Generator(device="cuda").manual_seed(n + k)
    rows = 2048
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w_next = torch.randn(k, n, device="cuda", generator=g) / n ** 0.5  # backward: (k_next, n) weight
    gz = torch.randn(rows, k, device="cuda", generator=g) * 1e-3
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    pf, pb, pf2 = weight_planes([(w, False), (w_next, True), (w, False)])
    assert torch.equal(pf, pf2)
    assert torch.equal(linear_tanh_x6(x, w, b, planes=pf), linear_tanh_x6(x, w, b))
    g1, d1 = linear_tanh_backward_x6(gz, w_next, y, planes=pb)
    g2, d2 = linear_tanh_backward_x6(gz, w_next, y)
    assert torch.equal(g1, g2) and torch.equal(d1, d2)
    if n == 256:
        wo, bo = torch.randn(2, 256, device="cuda", generator=g), torch.zeros(2, device="cuda")
        y1, o1 = linear_tanh_out_x6(x, w, b, wo, bo, planes=pf)
        y2, o2 = linear_tanh_out_x6(x, w, b, wo, bo)
        assert torch.equal(y1, y2) and torch.equal(o1, o2)


@pytest.mark.gpu
def test_weight_planes_refusals_gpu():
    from vss_amd.update import weight_planes
    w = torch.randn(256, 512, device="cuda")
    with pytest.raises(ValueError):
        weight_planes([])
    with pytest.raises(ValueError):
        weight_planes([(w, False)] * 17)  # at most 16 per launch
    with pytest.raises(N.NativeError):
        weight_planes([(torch.randn(100, 512, device="cuda"), False)])  # n % 128
    with pytest.raises(N.NativeError):
        weight_planes([(torch.randn(256, 100, device="cuda"), False)])  # k % 64
    with pytest.raises(ValueError):
        linear_tanh_x6(torch.randn(256, 512, device="cuda"), w, torch.zeros(256, device="cuda"),
                       planes=torch.empty(3, 10, device="cuda", dtype=torch.int16))
