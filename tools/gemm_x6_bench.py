#!/usr/bin/env python3
"""Profiling-only: the update's GEMMs on the bf16 matrix cores with fp32 arithmetic
(csrc/vss_gemm_x6.hip) against the fp32-MFMA kernels (csrc/vss_update.hip) and hipBLASLt's fp32 GEMM,
at the update's shapes (ROWS = 2,097,152 minibatch rows; the Agent's 256->512, 512->512, 512->256
layers).  Two parts:

  accuracy (ACC_ROWS rows): error of each path against an fp64 evaluation of the same function
  timing   (ROWS rows):     microseconds and TFLOP/s (fp32 FLOP of the GEMM) per launch

  forward   y = tanh(x W^T + b)            x6 vs vss_linear_tanh vs torch addmm + tanh
  backward  gz = (g W) * (1 - y^2), db     x6 vs vss_linear_tanh_backward vs torch mm + tanh_grad_bias
  wgrad     dW = g^T x                     x6 vs torch (hipBLASLt) mm
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import update as U  # noqa: E402


def timeit(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def err(out, ref64):
    d = (out.double() - ref64)
    return float(d.abs().max() / ref64.abs().max()), float(d.norm() / ref64.norm())


def operands(rows, k, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    gz = torch.randn(rows, n, device="cuda", generator=g) * 1e-3  # gradient w.r.t. this layer's output
    y_lo = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))  # the tanh output below (backward)
    return x, w, b, gz, y_lo


def accuracy(rows):
    print(f"accuracy vs fp64 at {rows} rows: max|err|/max|ref|, ||err||/||ref||", flush=True)
    for k, n in ((256, 512), (512, 512), (512, 256)):
        x, w, b, gz, y_lo = operands(rows, k, n, k * n)
        ref = torch.tanh(x.double() @ w.double().t() + b.double())
        print(f"FWD {k}->{n}: x6 {err(U.linear_tanh_x6(x, w, b), ref)}  fp32-mfma {err(U.linear_tanh(x, w, b), ref)}  "
              f"torch {err(torch.addmm(b, x, w.t()).tanh_(), ref)}", flush=True)
        # backward into the tanh below: gz (rows, n) through W (n, k) into y_lo (rows, k)
        ref = (gz.double() @ w.double()) * (1 - y_lo.double() ** 2)
        gx6, _ = U.linear_tanh_backward_x6(gz, w, y_lo)
        gf, _ = U.linear_tanh_backward(gz, w, y_lo)
        gt = gz.mm(w) * (1 - y_lo * y_lo)
        print(f"BWD {n}->{k}: x6 {err(gx6, ref)}  fp32-mfma {err(gf, ref)}  torch {err(gt, ref)}", flush=True)
        if U.x6_wgrad_ok(rows, n, k):
            ref = gz.double().t() @ x.double()
            print(f"WGRAD {n}x{k}: x6 {err(U.weight_grad_x6(gz, x), ref)}  torch {err(gz.t().mm(x), ref)}", flush=True)
        if n == 256:
            wo = torch.randn(2, 256, device="cuda") / 16
            bo = torch.randn(2, device="cuda") * 0.1
            yr = torch.tanh(x.double() @ w.double().t() + b.double())
            oref = yr @ wo.double().t() + bo.double()
            y6, o6 = U.linear_tanh_out_x6(x, w, b, wo, bo)
            yf, of = U.linear_tanh_out(x, w, b, wo, bo)
            print(f"FWD+OUT {k}->256->2: x6 y {err(y6, yr)} out {err(o6, oref)}  fp32-mfma y {err(yf, yr)} "
                  f"out {err(of, oref)}", flush=True)


def timing(rows):
    print(f"timing at {rows} rows (us per launch, fp32-equivalent TF)", flush=True)
    for k, n in ((256, 512), (512, 512), (512, 256)):
        x, w, b, gz, y_lo = operands(rows, k, n, 7)
        fl = 2.0 * rows * k * n
        t6 = timeit(lambda: U.linear_tanh_x6(x, w, b))
        tf = timeit(lambda: U.linear_tanh(x, w, b))
        print(f"FWD {k:3d}->{n:3d}: x6 {t6:7.0f} us {fl / t6 / 1e6:6.1f} TF | fp32-mfma {tf:7.0f} us "
              f"{fl / tf / 1e6:6.1f} TF", flush=True)
        t6 = timeit(lambda: U.linear_tanh_backward_x6(gz, w, y_lo))
        tf = timeit(lambda: U.linear_tanh_backward(gz, w, y_lo))
        print(f"BWD {n:3d}->{k:3d}: x6 {t6:7.0f} us {fl / t6 / 1e6:6.1f} TF | fp32-mfma {tf:7.0f} us "
              f"{fl / tf / 1e6:6.1f} TF", flush=True)
        if U.x6_wgrad_ok(rows, n, k):
            t6 = timeit(lambda: U.weight_grad_x6(gz, x))
            tt = timeit(lambda: gz.t().mm(x))
            print(f"WGRAD {n:3d}x{k:3d}: x6 {t6:7.0f} us {fl / t6 / 1e6:6.1f} TF | hipBLASLt {tt:7.0f} us "
                  f"{fl / tt / 1e6:6.1f} TF", flush=True)
        if n == 256:
            wo = torch.randn(2, 256, device="cuda") / 16
            bo = torch.randn(2, device="cuda") * 0.1
            t6 = timeit(lambda: U.linear_tanh_out_x6(x, w, b, wo, bo))
            tf = timeit(lambda: U.linear_tanh_out(x, w, b, wo, bo))
            print(f"FWD+OUT {k:3d}->256->2: x6 {t6:7.0f} us {fl / t6 / 1e6:6.1f} TF | fp32-mfma {tf:7.0f} us "
                  f"{fl / tf / 1e6:6.1f} TF", flush=True)
        del x, w, b, gz, y_lo
        torch.cuda.empty_cache()


if __name__ == "__main__":
    accuracy(int(os.environ.get("ACC_ROWS", 16384)))
    timing(int(os.environ.get("ROWS", 2097152)))
