"""PPO-update helpers (csrc/vss_update.hip, include/vss.h):

    gz, db = tanh_grad_bias(gy, y)                # gz = gy * (1 - y^2), db = gz.sum(0)
    y = linear_tanh(x, w, b)                      # tanh(x @ w.T + b)
    y, out = linear_tanh_out(x, w, b, w_o, b_o)   # the same plus the output layer y @ w_o.T + b_o
    gz, db = linear_tanh_backward(gz_next, w_next, y)
                                                  # gz = (gz_next @ w_next) * (1 - y^2), db = gz.sum(0)
    gz, db, dw = output_backward(g_out, w_out, y) # the same through the output layer, plus its
                                                  # weight gradient dw = g_out.T @ y, in one pass

They replace what autograd issues for the Agent's nn.Linear -> nn.Tanh pairs
(ppo_continuous_action_isaacgym.py:104-111): tanh_backward + the bias-gradient reduction
(vss_tanh_grad_bias), addmm + tanh (vss_linear_tanh: one fp32 MFMA GEMM with bias and tanh in its
epilogue), and the input-gradient GEMM of the layer above + tanh_backward + bias reduction
(vss_linear_tanh_backward: one fp32 MFMA GEMM with the tanh derivative and the column sums in its
epilogue), and for the output layer (1, 2 or 6 columns) that backward together with the output
layer's weight gradient as one streaming pass over y (vss_output_backward).  On a ROCm device they run the HIP kernels (and raise if the library is missing); CPU
tensors (the CPU test suite's PPO loop) take the same formulas in torch.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N

_COLS = (64, 128, 256, 512, 1024)


def tanh_grad_bias(gy: torch.Tensor, y: torch.Tensor):
    if gy.shape != y.shape or gy.dim() != 2:
        raise ValueError(f"gy {tuple(gy.shape)} and y {tuple(y.shape)} must be the same (rows, cols)")
    if gy.device.type != "cuda":
        gz = gy * (1.0 - y * y)
        return gz, gz.sum(0)
    rows, cols = y.shape
    if cols not in _COLS or gy.dtype != torch.float32 or y.dtype != torch.float32:
        raise ValueError(f"vss_tanh_grad_bias: fp32 with cols in {_COLS}, got {gy.dtype}/{y.dtype} x {cols}")
    lib = N.load()
    if rows == 0:  # empty tensors have no storage to hand over
        return torch.empty_like(y), torch.zeros(cols, device=y.device, dtype=torch.float32)
    gy = gy.contiguous()
    y = y.contiguous()
    gz = torch.empty_like(y)
    partial = torch.empty((lib.vss_tanh_grad_chunks(rows, cols), cols), device=y.device, dtype=torch.float32)
    N.check(lib.vss_tanh_grad_bias(N.stream_of(y.device), rows, cols, gy.data_ptr(), y.data_ptr(), gz.data_ptr(),
                                   partial.data_ptr()), "vss_tanh_grad_bias")
    return gz, partial.sum(0)


def gemm_shape_ok(k: int, n: int) -> bool:
    """Shapes the fused GEMMs take: contraction k % 4 == 0, output width n % 128 == 0."""
    return k >= 4 and k % 4 == 0 and n >= 128 and n % 128 == 0


def _fp32_2d(name, *ts):
    for t in ts:
        if t.dtype != torch.float32:
            raise ValueError(f"{name}: fp32 tensors only, got {t.dtype}")


def _out(out, shape, like):
    if out is None:
        return torch.empty(shape, device=like.device, dtype=torch.float32)
    if tuple(out.shape) != tuple(shape) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous fp32 {tuple(shape)} tensor, got {out.dtype} {tuple(out.shape)}")
    return out


SUM_PARTS_MAX = 512


def _reduce_parts(parts: torch.Tensor, out: torch.Tensor | None, defer: list | None) -> torch.Tensor:
    """The sum over dim 0 of a kernel's partial results, into `out` when given; with a `defer` list the
    reduction is queued there for ONE sum_parts launch later (into `out`, or a new tensor returned now and
    filled by that launch: the caller reads it only after running the list).  Parts lists longer than
    SUM_PARTS_MAX (the output layer's 2,048 streaming-block partials) stay on torch.sum, whose reduction
    splits the parts over many blocks (sum_parts gives each output element one block's 4 waves: 2,048
    parts made the launch 243 us instead of 34, profiles/r05i_*)."""
    if defer is not None and parts.is_cuda and parts.shape[0] <= SUM_PARTS_MAX:
        if out is None:
            out = torch.empty(parts.shape[1:], device=parts.device, dtype=torch.float32)
        defer.append((parts, out))
        return out
    return torch.sum(parts, 0, out=out)


def sum_parts(jobs) -> None:
    """jobs = [(parts (S, ...) fp32, out (...) fp32)]: out = parts.sum(0) for all of them in one launch
    per 32 jobs (vss_sum_parts; parts summed in order s = 0 .. S-1, deterministic).  `out` may be a
    row-strided 2-D view; the last dim of both must be contiguous."""
    # the longest part lists first: their blocks (the longest serial chains) start first
    jobs = sorted(jobs, key=lambda j: -j[0].shape[0])
    for q0 in range(0, len(jobs), 32):
        chunk = jobs[q0:q0 + 32]
        cols = {k: [] for k in ("src", "dst", "parts", "pstride", "rows", "cols", "sld", "dld")}
        for parts, out in chunk:
            # views only: a reshape that had to copy would hand the launch below a temporary's address
            try:
                p3 = parts.view(parts.shape[0], -1, parts.shape[-1]) if parts.dim() >= 2 else None
                o2 = out.view(1, -1) if out.dim() == 1 else out
            except RuntimeError as e:
                raise ValueError(f"sum_parts: parts {tuple(parts.shape)} / out {tuple(out.shape)} are not "
                                 f"viewable in the launch's shape ({e})") from None
            if p3 is None or parts.dtype != torch.float32 or out.dtype != torch.float32 or o2.dim() != 2 \
                    or tuple(p3.shape[1:]) != tuple(o2.shape) or p3.stride(2) != 1 or o2.stride(1) != 1 \
                    or not parts.is_cuda or out.device != parts.device:
                raise ValueError(f"sum_parts: parts {tuple(parts.shape)} / out {tuple(out.shape)}")
            cols["src"].append(p3.data_ptr())
            cols["dst"].append(o2.data_ptr())
            cols["parts"].append(p3.shape[0])
            cols["pstride"].append(p3.stride(0))
            cols["rows"].append(o2.shape[0])
            cols["cols"].append(o2.shape[1])
            cols["sld"].append(p3.stride(1) if o2.shape[0] > 1 else o2.shape[1])
            cols["dld"].append(o2.stride(0) if o2.shape[0] > 1 else o2.shape[1])
        c = len(chunk)
        Pa, I64 = ctypes.c_void_p * c, ctypes.c_int64 * c
        N.check(N.load().vss_sum_parts(N.stream_of(chunk[0][0].device), c, Pa(*cols["src"]), Pa(*cols["dst"]),
                                       I64(*cols["parts"]), I64(*cols["pstride"]), I64(*cols["rows"]),
                                       I64(*cols["cols"]), I64(*cols["sld"]), I64(*cols["dld"])), "vss_sum_parts")


def linear_tanh(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """tanh(x @ w.T + b) for x (rows, k), w (n, k) (nn.Linear's weight), b (n,)."""
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1] or b.shape != (w.shape[0],):
        raise ValueError(f"linear_tanh: x {tuple(x.shape)}, w {tuple(w.shape)}, b {tuple(b.shape)}")
    if x.device.type != "cuda":
        return torch.addmm(b, x, w.t()).tanh_()
    rows, k = x.shape
    n = w.shape[0]
    _fp32_2d("vss_linear_tanh", x, w, b)
    if not gemm_shape_ok(k, n):
        raise ValueError(f"vss_linear_tanh: k % 4 == 0 and n % 128 == 0 required, got k={k}, n={n}")
    lib = N.load()
    y = _out(out, (rows, n), x)
    if rows == 0:
        return y
    x, w, b = x.contiguous(), w.contiguous(), b.contiguous()
    N.check(lib.vss_linear_tanh(N.stream_of(x.device), rows, k, n, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                y.data_ptr()), "vss_linear_tanh")
    return y


def linear_tanh_out_ok(rows: int, k: int, n: int, k_out: int) -> bool:
    """Shapes vss_linear_tanh_out takes (the last hidden layer of the Agent's MLPs at the update's
    minibatch sizes): n = 256, rows % 256 == 0, k % 64 == 0, k_out in {1, 2, 6}."""
    return n == 256 and rows > 0 and rows % 256 == 0 and k % 64 == 0 and k_out in (1, 2, 6)


def linear_tanh_out(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, w_out: torch.Tensor, b_out: torch.Tensor):
    """(y, out): y = tanh(x @ w.T + b) and out = y @ w_out.T + b_out (the output nn.Linear) from ONE
    launch: the output layer's partial sums come from the GEMM's epilogue (vss_linear_tanh_out)."""
    rows, k = x.shape
    n, k_out = w.shape[0], w_out.shape[0]
    if x.device.type != "cuda":
        y = torch.addmm(b, x, w.t()).tanh_()
        return y, torch.addmm(b_out, y, w_out.t())
    if w.shape != (n, k) or b.shape != (n,) or w_out.shape != (k_out, n) or b_out.shape != (k_out,) \
            or not linear_tanh_out_ok(rows, k, n, k_out):
        raise ValueError(f"linear_tanh_out: x {tuple(x.shape)}, w {tuple(w.shape)}, w_out {tuple(w_out.shape)}")
    _fp32_2d("vss_linear_tanh_out", x, w, b, w_out, b_out)
    x, w, b, w_out = x.contiguous(), w.contiguous(), b.contiguous(), w_out.contiguous()
    y = torch.empty((rows, n), device=x.device, dtype=torch.float32)
    part = torch.empty((n // 64, rows, k_out), device=x.device, dtype=torch.float32)
    N.check(N.load().vss_linear_tanh_out(N.stream_of(x.device), rows, k, n, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                         y.data_ptr(), k_out, w_out.data_ptr(), part.data_ptr()), "vss_linear_tanh_out")
    return y, part.sum(0).add_(b_out)


def linear_tanh_backward(gz_next: torch.Tensor, w_next: torch.Tensor, y: torch.Tensor, out: torch.Tensor | None = None):
    """The pre-activation gradient of a tanh layer from the one of the layer above:
    gz = (gz_next @ w_next) * (1 - y^2) and db = gz.sum(0), with gz_next (rows, k_next), w_next
    (k_next, n) (the next layer's nn.Linear weight), y (rows, n) (this layer's tanh output)."""
    if gz_next.dim() != 2 or w_next.dim() != 2 or y.dim() != 2 or gz_next.shape[0] != y.shape[0] \
            or w_next.shape != (gz_next.shape[1], y.shape[1]):
        raise ValueError(f"linear_tanh_backward: gz_next {tuple(gz_next.shape)}, w_next {tuple(w_next.shape)}, "
                         f"y {tuple(y.shape)}")
    if gz_next.device.type != "cuda":
        gz = gz_next.mm(w_next) * (1.0 - y * y)
        return gz, gz.sum(0)
    rows, k_next = gz_next.shape
    n = y.shape[1]
    _fp32_2d("vss_linear_tanh_backward", gz_next, w_next, y)
    if not gemm_shape_ok(k_next, n):
        raise ValueError(f"vss_linear_tanh_backward: k_next % 4 == 0 and n % 128 == 0 required, got {k_next}, {n}")
    lib = N.load()
    gz = _out(out, (rows, n), y)
    if rows == 0:
        return gz, torch.zeros(n, device=y.device, dtype=torch.float32)
    gz_next, y = gz_next.contiguous(), y.contiguous()
    w_t = w_next.t().contiguous()  # (n, k_next): the kernel's K-contiguous operand layout
    partial = torch.empty((lib.vss_linear_tanh_backward_chunks(rows, k_next, n), n), device=y.device,
                          dtype=torch.float32)
    N.check(lib.vss_linear_tanh_backward(N.stream_of(y.device), rows, k_next, n, gz_next.data_ptr(), w_t.data_ptr(),
                                         y.data_ptr(), gz.data_ptr(), partial.data_ptr()),
            "vss_linear_tanh_backward")
    return gz, partial.sum(0)


def output_backward_ok(k_out: int, n: int) -> bool:
    """Shapes vss_output_backward takes: k_out <= 8 output columns over a layer of width n | 1024."""
    return 1 <= k_out <= 8 and n >= 128 and n % 128 == 0 and 1024 % n == 0


def output_backward(g_out: torch.Tensor, w_out: torch.Tensor, y: torch.Tensor, out_db: torch.Tensor | None = None,
                    out_dw: torch.Tensor | None = None, defer: list | None = None):
    """Backward through the output nn.Linear (weight w_out (k_out, n)) into the tanh layer below it
    (output y (rows, n), also the output layer's input), g_out (rows, k_out) the output's gradient:
    gz = (g_out @ w_out) * (1 - y^2), db = gz.sum(0) and dw = g_out.T @ y (the output layer's weight
    gradient).  out_db / out_dw: where to reduce db / dw into (ROCm path; the same tensors returned)."""
    if g_out.dim() != 2 or w_out.dim() != 2 or y.dim() != 2 or g_out.shape[0] != y.shape[0] \
            or w_out.shape != (g_out.shape[1], y.shape[1]):
        raise ValueError(f"output_backward: g_out {tuple(g_out.shape)}, w_out {tuple(w_out.shape)}, y {tuple(y.shape)}")
    if g_out.device.type != "cuda":
        gz = g_out.mm(w_out) * (1.0 - y * y)
        return gz, gz.sum(0), g_out.t().mm(y)
    rows, k_out = g_out.shape
    n = y.shape[1]
    _fp32_2d("vss_output_backward", g_out, w_out, y)
    if not output_backward_ok(k_out, n):
        raise ValueError(f"vss_output_backward: k_out <= 8 and n in (128, 256, 512, 1024) required, got {k_out}, {n}")
    lib = N.load()
    k_pad = 4 if k_out <= 4 else 8
    gz = torch.empty((rows, n), device=y.device, dtype=torch.float32)
    if rows == 0:
        z = torch.zeros(n, device=y.device, dtype=torch.float32)
        return gz, z, torch.zeros((k_out, n), device=y.device, dtype=torch.float32)
    g_pad = torch.nn.functional.pad(g_out, (0, k_pad - k_out)).contiguous()
    w_t = torch.nn.functional.pad(w_out, (0, 0, 0, k_pad - k_out)).t().contiguous()  # (n, k_pad)
    y = y.contiguous()
    chunks = lib.vss_output_backward_chunks(rows, k_pad, n)
    bpart = torch.empty((chunks, n), device=y.device, dtype=torch.float32)
    wpart = torch.empty((chunks, k_pad, n), device=y.device, dtype=torch.float32)
    N.check(lib.vss_output_backward(N.stream_of(y.device), rows, k_pad, n, g_pad.data_ptr(), w_t.data_ptr(),
                                    y.data_ptr(), gz.data_ptr(), bpart.data_ptr(), wpart.data_ptr()),
            "vss_output_backward")
    return gz, _reduce_parts(bpart, out_db, defer), _reduce_parts(wpart[:, :k_out], out_dw, defer)


def output_backward_direct_ok(k_out: int, n: int) -> bool:
    """Shapes vss_output_backward_direct takes: k_out in {1, 2, 3, 4, 6, 8}, n in {128, 256, 512, 1024}."""
    return k_out in (1, 2, 3, 4, 6, 8) and n >= 128 and n % 128 == 0 and 1024 % n == 0


def output_backward_direct(g_out: torch.Tensor, w_out: torch.Tensor, y: torch.Tensor, out_db: torch.Tensor | None = None,
                           out_dw: torch.Tensor | None = None, defer: list | None = None):
    """output_backward for the update's minibatch without autograd (vss_output_backward_direct): g_out
    (rows, k_out) and w_out (k_out, n) as they are (no padded copies), at most 256 partial rows, so the
    bias and weight gradients join the backward's sum_parts launch (defer).  Returns (gz, db, dw)."""
    rows, k_out = g_out.shape
    n = y.shape[1]
    if w_out.shape != (k_out, n) or y.shape[0] != rows or not output_backward_direct_ok(k_out, n):
        raise ValueError(f"output_backward_direct: g_out {tuple(g_out.shape)}, w_out {tuple(w_out.shape)}, y {tuple(y.shape)}")
    _x6_check("vss_output_backward_direct", True, g_out, w_out, y)
    lib = N.load()
    g_out, w_out, y = g_out.contiguous(), w_out.contiguous(), y.contiguous()
    gz = torch.empty((rows, n), device=y.device, dtype=torch.float32)
    chunks = lib.vss_output_backward_direct_chunks(rows, k_out, n)
    bpart = torch.empty((max(chunks, 1), n), device=y.device, dtype=torch.float32)
    wpart = torch.empty((max(chunks, 1), k_out, n), device=y.device, dtype=torch.float32)
    if rows == 0:
        bpart.zero_()
        wpart.zero_()
    N.check(lib.vss_output_backward_direct(N.stream_of(y.device), rows, k_out, n, g_out.data_ptr(), w_out.data_ptr(),
                                           y.data_ptr(), gz.data_ptr(), bpart.data_ptr(), wpart.data_ptr()),
            "vss_output_backward_direct")
    return gz, _reduce_parts(bpart, out_db, defer), _reduce_parts(wpart, out_dw, defer)


def linear_tanh_loss_x6_ok(rows_pad: int, k: int, n: int, k_out: int) -> bool:
    """Shapes vss_linear_tanh_loss_bf16x6 takes: a 256-wide last hidden layer on the x6 shapes, 1 or 2
    outputs."""
    return n == 256 and k_out in (1, 2) and x6_ok(rows_pad, k, n)


def linear_tanh_loss_x6(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, w_out: torch.Tensor, b_out: torch.Tensor,
                        rows: int, actor: bool, *, planes: torch.Tensor | None = None, act=None, logp=None, adv=None,
                        adv_part=None, adv_count: float = 0.0, logstd=None, ret=None, val=None, clip_coef: float = 0.2,
                        vf_coef: float = 0.5, clip_vloss: bool = False, out_db=None, out_dw=None, defer=None):
    """The last hidden layer, the output layer, one network's loss terms and the output layer's backward
    in ONE x6 launch (vss_linear_tanh_loss_bf16x6, direct_minibatch): x (rows_pad, k) the layer's input,
    w (256, k) / b its weight and bias (planes: weight_planes() of w, or None to split it here), w_out /
    b_out the output layer's; actor: act / logp / adv (RAW, normalised from adv_part over adv_count as
    ppo_loss_direct) / logstd, else ret / val.  Returns (gz (rows_pad, 256) the hidden layer's
    pre-activation gradient, its bias gradient, the output weight's gradient (both into out_db / out_dw,
    summed through `defer` when given), the per-block loss sums for ppo_loss_fused_finish)."""
    rows_pad, k = x.shape
    n, k_out = w.shape[0], w_out.shape[0]
    _x6_check("vss_linear_tanh_loss_bf16x6", w.shape == (n, k) and b.shape == (n,) and w_out.shape == (k_out, n)
              and b_out.shape == (k_out,) and 0 < rows <= rows_pad and linear_tanh_loss_x6_ok(rows_pad, k, n, k_out)
              and (actor or k_out == 1), x, w, b, w_out)
    rows_t = (act, logp, adv, logstd) if actor else (ret,) + ((val,) if clip_vloss else ())
    for t in rows_t:
        if t is None or t.dtype != torch.float32 or t.device != x.device or not t.is_contiguous():
            raise ValueError("linear_tanh_loss_x6: the role's loss inputs as contiguous fp32 tensors on the device")
    if actor and (act.shape[0] < rows_pad or act.shape[1] != k_out or logp.shape[0] < rows or adv.shape[0] < rows
                  or logstd.numel() != k_out):
        raise ValueError(f"linear_tanh_loss_x6: actor inputs for {rows} rows and {k_out} actions")
    if not actor and (ret.shape[0] < rows or (clip_vloss and val.shape[0] < rows)):
        raise ValueError(f"linear_tanh_loss_x6: critic inputs for {rows} rows")
    if adv_part is not None and (adv_part.dtype != torch.float64 or adv_part.device != x.device
                                 or adv_part.dim() != 2 or adv_part.shape[1] != 2 or not adv_part.is_contiguous()):
        raise ValueError("linear_tanh_loss_x6: adv_part must be a contiguous (parts, 2) fp64 tensor on the device")
    lib = N.load()
    x, b, w_out, b_out = x.contiguous(), b.contiguous(), w_out.contiguous(), b_out.contiguous()
    if planes is None:  # the fused entry takes only the planes
        planes = weight_planes([(w.contiguous(), False)])[0]
    _, pp, keep = _w_and_planes(w, planes)
    blocks = lib.vss_linear_tanh_loss_blocks_bf16x6(rows_pad, k, n)
    f32 = dict(device=x.device, dtype=torch.float32)
    gz = torch.empty((rows_pad, n), **f32)
    part_cs = torch.empty((blocks, n), **f32)
    part_dw = torch.empty((blocks, k_out, n), **f32)
    stats = torch.empty((blocks, 32), **f32)
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    c = float(clip_coef)
    N.check(lib.vss_linear_tanh_loss_bf16x6(
        N.stream_of(x.device), 0 if actor else 1, rows_pad, rows, k, n, x.data_ptr(), b.data_ptr(), k_out,
        w_out.data_ptr(), b_out.data_ptr(), ptr(act), ptr(logp), ptr(adv), ptr(adv_part),
        adv_part.shape[0] if adv_part is not None else 0, float(adv_count), ptr(logstd), ptr(ret),
        ptr(val) if clip_vloss else None, c, 1 - c, 1 + c, float(vf_coef), int(bool(clip_vloss)), gz.data_ptr(),
        part_cs.data_ptr(), part_dw.data_ptr(), stats.data_ptr(), pp), "vss_linear_tanh_loss_bf16x6")
    del keep
    return gz, _reduce_parts(part_cs, out_db, defer), _reduce_parts(part_dw, out_dw, defer), stats


# ---- the same GEMMs in fp32 arithmetic on the bf16 matrix cores (csrc/vss_gemm_x6.hip) ----------------
# Every operand is split exactly into three bf16 parts and each product is summed from the six partial
# products above 2^-23 |a||b| in fp32 (tests/test_gemm_x6.py: the error is that of an fp32 GEMM).
# Exact shapes only; the callers keep the fp32-MFMA entries above for the others.

def x6_ok(rows: int, k: int, n: int) -> bool:
    """Shapes the bf16x6 forward / backward take: rows % 256, n % 128, k % 64."""
    return rows > 0 and rows % 256 == 0 and n > 0 and n % 128 == 0 and n <= 4096 and k > 0 and k % 64 == 0


def x6_wgrad_ok(rows: int, n_out: int, k_in: int) -> bool:
    """Shapes the bf16x6 weight gradient takes: rows % 64, n_out % 256, k_in % 128."""
    return rows > 0 and rows % 64 == 0 and n_out % 256 == 0 and 0 < n_out <= 4096 and k_in % 128 == 0 \
        and 0 < k_in <= 4096


def _planes(w: torch.Tensor) -> torch.Tensor:
    """Scratch for a weight's three bf16 planes (the x6 entry points fill it before their GEMM)."""
    return torch.empty((3, w.numel()), device=w.device, dtype=torch.int16)


def weight_planes(jobs) -> list:
    """The bf16 planes of several weights in ONE launch (vss_weight_planes_bf16x6): jobs = [(w, transpose)]
    with w an fp32 (n, k) weight (transpose False: the forward's P operand) or a (k, n) one whose
    transpose is the operand (True: the backward's W_next^T, no transposed copy); at most 8.  Returns
    the planes (at most 16 jobs), to be handed to linear_tanh_x6 / linear_tanh_out_x6 / linear_tanh_backward_x6 (planes=),
    valid until the weights change."""
    if not 1 <= len(jobs) <= 16:
        raise ValueError(f"weight_planes: 1..16 weights per launch, got {len(jobs)}")
    ws, ns, ks, ts, outs = [], [], [], [], []
    for w, tr in jobs:
        if w.dim() != 2 or w.dtype != torch.float32 or not w.is_cuda or not w.is_contiguous():
            raise ValueError(f"weight_planes: contiguous fp32 ROCm (rows, cols) weights, got {w.dtype} {tuple(w.shape)}")
        n, k = (w.shape[1], w.shape[0]) if tr else (w.shape[0], w.shape[1])
        ws.append(w.data_ptr())
        ns.append(n)
        ks.append(k)
        ts.append(int(bool(tr)))
        outs.append(_planes(w))
    c = len(jobs)
    P, I = ctypes.c_void_p * c, ctypes.c_int32 * c
    N.check(N.load().vss_weight_planes_bf16x6(N.stream_of(jobs[0][0].device), c, P(*ws), I(*ns), I(*ks), I(*ts),
                                              P(*[o.data_ptr() for o in outs])), "vss_weight_planes_bf16x6")
    return outs


def _x6_check(name, cond, *ts):
    if not cond:
        raise ValueError(f"{name}: shape outside the bf16x6 kernels' exact shapes: {[tuple(t.shape) for t in ts]}")
    _fp32_2d(name, *ts)
    for t in ts:
        if t.device.type != "cuda":
            raise ValueError(f"{name}: ROCm tensors only (no CPU path)")


def _w_and_planes(w: torch.Tensor, planes: torch.Tensor | None):
    """(weight pointer, planes pointer, keep) for an x6 entry: the entry splits w itself (planes None),
    or takes the weight_planes() result with a NULL weight.  `keep` holds the tensors behind the pointers
    (w, e.g. a transposed copy, and the planes scratch): the caller keeps it until its launch is queued,
    so that no allocation in between (the output, the partial sums) can take their memory while the
    split and the GEMM still use it."""
    if planes is None:
        scratch = _planes(w)
        return w.data_ptr(), scratch.data_ptr(), (w, scratch)
    if planes.dtype != torch.int16 or planes.numel() != 3 * w.numel():
        raise ValueError(f"planes: weight_planes() output of this weight, got {planes.dtype} {tuple(planes.shape)}")
    return None, planes.data_ptr(), (planes,)


def linear_tanh_x6(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                   planes: torch.Tensor | None = None) -> torch.Tensor:
    """linear_tanh on the bf16 matrix cores with fp32 arithmetic (vss_linear_tanh_bf16x6); planes: w's
    weight_planes() (transpose False), or None to split w in the call."""
    rows, k = x.shape
    n = w.shape[0]
    _x6_check("vss_linear_tanh_bf16x6", w.shape == (n, k) and b.shape == (n,) and x6_ok(rows, k, n), x, w, b)
    x, w, b = x.contiguous(), w.contiguous(), b.contiguous()
    y = _out(out, (rows, n), x)
    wp, pp, keep = _w_and_planes(w, planes)
    N.check(N.load().vss_linear_tanh_bf16x6(N.stream_of(x.device), rows, k, n, x.data_ptr(), wp,
                                            b.data_ptr(), y.data_ptr(), pp), "vss_linear_tanh_bf16x6")
    del keep  # the split and the GEMM are queued: the scratch may be reused from here on
    return y


def linear_tanh_out_x6(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, w_out: torch.Tensor, b_out: torch.Tensor,
                       out: torch.Tensor | None = None, planes: torch.Tensor | None = None, parts: bool = False):
    """linear_tanh_out on the bf16 matrix cores with fp32 arithmetic (vss_linear_tanh_out_bf16x6).
    parts: return (y, the output layer's epilogue parts (n // 64, rows, k_out)) without summing them or
    adding b_out -- vss_ppo_loss_direct reads them as they are."""
    rows, k = x.shape
    n, k_out = w.shape[0], w_out.shape[0]
    _x6_check("vss_linear_tanh_out_bf16x6", w.shape == (n, k) and b.shape == (n,) and w_out.shape == (k_out, n)
              and b_out.shape == (k_out,) and n == 256 and k_out in (1, 2, 6) and x6_ok(rows, k, n), x, w, b, w_out)
    x, w, b, w_out = x.contiguous(), w.contiguous(), b.contiguous(), w_out.contiguous()
    y = _out(out, (rows, n), x)
    part = torch.empty((n // 64, rows, k_out), device=x.device, dtype=torch.float32)
    wp, pp, keep = _w_and_planes(w, planes)
    N.check(N.load().vss_linear_tanh_out_bf16x6(N.stream_of(x.device), rows, k, n, x.data_ptr(), wp,
                                                b.data_ptr(), y.data_ptr(), k_out, w_out.data_ptr(), part.data_ptr(),
                                                pp), "vss_linear_tanh_out_bf16x6")
    del keep  # the split and the GEMM are queued: the scratch may be reused from here on
    if parts:
        return y, part
    return y, part.sum(0).add_(b_out)


def linear_tanh_backward_x6(gz_next: torch.Tensor, w_next: torch.Tensor, y: torch.Tensor,
                            out: torch.Tensor | None = None, out_db: torch.Tensor | None = None,
                            planes: torch.Tensor | None = None, defer: list | None = None):
    """linear_tanh_backward on the bf16 matrix cores with fp32 arithmetic (vss_linear_tanh_backward_bf16x6);
    planes: w_next's weight_planes() with transpose True, or None to transpose and split it in the call."""
    rows, k_next = gz_next.shape
    n = y.shape[1]
    _x6_check("vss_linear_tanh_backward_bf16x6", w_next.shape == (k_next, n) and y.shape[0] == rows
              and x6_ok(rows, k_next, n), gz_next, w_next, y)
    lib = N.load()
    gz_next, y = gz_next.contiguous(), y.contiguous()
    if planes is None:
        wp, pp, keep = _w_and_planes(w_next.t().contiguous(), None)  # (n, k_next): K-contiguous
    else:
        wp, pp, keep = _w_and_planes(w_next, planes)
    gz = _out(out, (rows, n), y)
    partial = torch.empty((lib.vss_linear_tanh_backward_chunks_bf16x6(rows, k_next, n), n), device=y.device,
                          dtype=torch.float32)
    N.check(lib.vss_linear_tanh_backward_bf16x6(N.stream_of(y.device), rows, k_next, n, gz_next.data_ptr(),
                                                wp, y.data_ptr(), gz.data_ptr(), partial.data_ptr(), pp),
            "vss_linear_tanh_backward_bf16x6")
    del keep  # the split and the GEMM are queued: the scratch may be reused from here on
    return gz, _reduce_parts(partial, out_db, defer)


def weight_grad_x6(grad: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
                   defer: list | None = None) -> torch.Tensor:
    """dW = grad.T @ x (a Linear layer's weight gradient, grad (rows, n_out), x (rows, k_in)) on the
    bf16 matrix cores with fp32 arithmetic, split over the rows (vss_weight_grad_bf16x6); the parts are
    reduced into `out` when given."""
    rows, n_out = grad.shape
    k_in = x.shape[1]
    _x6_check("vss_weight_grad_bf16x6", x.shape[0] == rows and x6_wgrad_ok(rows, n_out, k_in), grad, x)
    lib = N.load()
    grad, x = grad.contiguous(), x.contiguous()
    parts = torch.empty((lib.vss_weight_grad_chunks_bf16x6(rows, n_out, k_in), n_out, k_in), device=x.device,
                        dtype=torch.float32)
    N.check(lib.vss_weight_grad_bf16x6(N.stream_of(x.device), rows, n_out, k_in, grad.data_ptr(), x.data_ptr(),
                                       parts.data_ptr()), "vss_weight_grad_bf16x6")
    return _reduce_parts(parts, out, defer)


def first_layer_x6_ok(k: int, n: int) -> bool:
    """Shapes vss_first_layer_bf16x6 takes (the Agent's first layer): n 256, k <= 64 and k % 4 == 0."""
    return n == 256 and 0 < k <= 64 and k % 4 == 0


def first_layer_x6(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """tanh(x @ w.T + b) for the Agent's first layer (x (rows, k <= 64) the observations, w (256, k)) on the
    bf16 matrix cores with fp32 arithmetic (vss_first_layer_bf16x6), any row count."""
    rows, k = x.shape
    n = w.shape[0]
    _x6_check("vss_first_layer_bf16x6", w.shape == (n, k) and b.shape == (n,) and first_layer_x6_ok(k, n), x, w, b)
    x, w, b = x.contiguous(), w.contiguous(), b.contiguous()
    y = _out(out, (rows, n), x)
    N.check(N.load().vss_first_layer_bf16x6(N.stream_of(x.device), rows, k, n, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                            y.data_ptr()), "vss_first_layer_bf16x6")
    return y


def first_wgrad_ok(rows: int, n_out: int, k_in: int) -> bool:
    """Shapes vss_first_weight_grad_bf16x6 takes (the Agent's first layer): n_out 256, k_in <= 64 and
    k_in % 4 == 0, rows % 64."""
    return rows > 0 and rows % 64 == 0 and n_out == 256 and 0 < k_in <= 64 and k_in % 4 == 0


def first_weight_grad_x6(grad: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
                         defer: list | None = None) -> torch.Tensor:
    """dW = grad.T @ x for the Agent's first layer (grad (rows, 256), x (rows, k_in <= 64): the
    observations) on the bf16 matrix cores with fp32 arithmetic, split over the rows
    (vss_first_weight_grad_bf16x6); the parts are reduced into `out` when given."""
    rows, n_out = grad.shape
    k_in = x.shape[1]
    _x6_check("vss_first_weight_grad_bf16x6", x.shape[0] == rows and first_wgrad_ok(rows, n_out, k_in), grad, x)
    lib = N.load()
    grad, x = grad.contiguous(), x.contiguous()
    parts = torch.empty((lib.vss_first_weight_grad_chunks_bf16x6(rows, n_out, k_in), n_out, k_in), device=x.device,
                        dtype=torch.float32)
    N.check(lib.vss_first_weight_grad_bf16x6(N.stream_of(x.device), rows, n_out, k_in, grad.data_ptr(), x.data_ptr(),
                                             parts.data_ptr()), "vss_first_weight_grad_bf16x6")
    return _reduce_parts(parts, out, defer)


# ---- any row count: whole tiles on the bf16x6 kernels, the ragged rest on the fp32 ones --------------
# The reference's default PPO shapes are not tile multiples (4,095 envs x 128 steps / 4 minibatches =
# 131,040 rows): the first rows // 256 * 256 rows (// 64 * 64 for the weight gradient) go to the x6
# kernels, the remaining < 256 (< 64) rows to hipBLASLt (torch addmm / mm, plain fp32 GEMMs) into the
# same output -- a persistent kernel on one or two row tiles would run latency-bound (the masked
# fp32-MFMA kernels took 120-128 us on a 224-row tail, profiles/r03r_*).

def linear_tanh_mixed(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, planes: torch.Tensor | None = None) -> torch.Tensor:
    rows, k = x.shape
    n = w.shape[0]
    if x.is_cuda and rows > 0 and first_layer_x6_ok(k, n):
        return first_layer_x6(x, w, b)  # the first layer (52 -> 256): every row on the bf16 matrix cores
    main = rows // 256 * 256
    if main == 0 or not x6_ok(main, k, n):
        return linear_tanh(x, w, b)
    y = torch.empty((rows, n), device=x.device, dtype=torch.float32)
    linear_tanh_x6(x[:main], w, b, out=y[:main], planes=planes)
    if main < rows:
        torch.addmm(b, x[main:], w.t(), out=y[main:]).tanh_()
    return y


def linear_tanh_out_mixed(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, w_out: torch.Tensor, b_out: torch.Tensor,
                          planes: torch.Tensor | None = None):
    rows, k = x.shape
    n, k_out = w.shape[0], w_out.shape[0]
    main = rows // 256 * 256
    if main == 0 or not x6_ok(main, k, n) or n != 256 or k_out not in (1, 2, 6):
        y = linear_tanh(x, w, b)
        return y, torch.addmm(b_out, y, w_out.t())
    y = torch.empty((rows, n), device=x.device, dtype=torch.float32)
    _, o_main = linear_tanh_out_x6(x[:main], w, b, w_out, b_out, out=y[:main], planes=planes)
    if main == rows:
        return y, o_main
    y_t = torch.addmm(b, x[main:], w.t(), out=y[main:]).tanh_()
    return y, torch.cat([o_main, torch.addmm(b_out, y_t, w_out.t())])


def linear_tanh_backward_mixed(gz_next: torch.Tensor, w_next: torch.Tensor, y: torch.Tensor,
                               out_db: torch.Tensor | None = None, planes: torch.Tensor | None = None,
                               defer: list | None = None):
    """out_db: where to reduce the bias gradient into (the same tensor returned); planes: w_next's
    weight_planes() with transpose True (None: split in the call); defer: queue the bias reduction
    (_reduce_parts) when the rows are whole tiles."""
    rows, k_next = gz_next.shape
    n = y.shape[1]
    main = rows // 256 * 256
    if main == 0 or not x6_ok(main, k_next, n):
        gz, db = linear_tanh_backward(gz_next, w_next, y)
        return gz, (db if out_db is None else out_db.copy_(db))
    gz = torch.empty((rows, n), device=y.device, dtype=torch.float32)
    _, db = linear_tanh_backward_x6(gz_next[:main], w_next, y[:main], out=gz[:main], out_db=out_db, planes=planes,
                                    defer=defer if main == rows else None)
    if main < rows:
        y_t = y[main:]
        gz_t = torch.mm(gz_next[main:], w_next, out=gz[main:]).mul_(1.0 - y_t * y_t)
        db = db.add_(gz_t.sum(0)) if out_db is not None else db + gz_t.sum(0)
    return gz, db


def weight_grad_mixed(grad: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
                      defer: list | None = None) -> torch.Tensor:
    """out: where to reduce the weight gradient into (the same tensor returned).  The hidden layers'
    shapes on vss_weight_grad_bf16x6, the first layer's (x = the observations) on
    vss_first_weight_grad_bf16x6."""
    rows, n_out = grad.shape
    k_in = x.shape[1]
    main = rows // 64 * 64
    if main > 0 and first_wgrad_ok(main, n_out, k_in):
        fn = first_weight_grad_x6
    elif main > 0 and x6_wgrad_ok(main, n_out, k_in):
        fn = weight_grad_x6
    else:
        return torch.mm(grad.t(), x, out=out)
    dw = fn(grad[:main], x[:main], out=out, defer=defer if main == rows else None)
    if main < rows:
        dw = dw.addmm_(grad[main:].t(), x[main:])
    return dw
