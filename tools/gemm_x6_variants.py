#!/usr/bin/env python3
"""Profiling-only: A/B of builds of csrc/vss_gemm_x6.hip at the update's shapes (ROWS = 2,097,152).
The product library and every tools/_build/libx6_<name>.so are timed in interleaved rounds (median
of ROUNDS); names starting with "old_" use the entry points without the w_split scratch."""
import ctypes
import glob
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import _native as N  # noqa: E402


def libs():
    out = [("product", N.load(), False)]
    for path in sorted(glob.glob(os.path.join(REPO, "tools", "_build", "libx6_*.so"))):
        name = os.path.basename(path)[6:-3]
        L = ctypes.CDLL(path)
        old = name.startswith("old_")
        P, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.vss_linear_tanh_bf16x6.argtypes = [P, i64, i32, i32] + [P] * (4 if old else 5)
        L.vss_linear_tanh_backward_chunks_bf16x6.argtypes = [i64, i32, i32]
        L.vss_linear_tanh_backward_chunks_bf16x6.restype = i64
        L.vss_linear_tanh_backward_bf16x6.argtypes = [P, i64, i32, i32] + [P] * (5 if old else 6)
        L.vss_weight_grad_chunks_bf16x6.argtypes = [i64, i32, i32]
        L.vss_weight_grad_chunks_bf16x6.restype = i64
        L.vss_weight_grad_bf16x6.argtypes = [P, i64, i32, i32, P, P, P]
        out.append((name, L, old))
    return out


def timeit(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    rows = int(os.environ.get("ROWS", 2097152))
    rounds = int(os.environ.get("ROUNDS", 3))
    st = torch.cuda.current_stream().cuda_stream
    L = libs()
    g = torch.Generator(device="cuda").manual_seed(1)
    a512 = torch.tanh(torch.randn(rows, 512, device="cuda", generator=g))
    b512 = torch.randn(rows, 512, device="cuda", generator=g) * 1e-3
    c256 = torch.tanh(torch.randn(rows, 256, device="cuda", generator=g))
    out = torch.empty(rows, 512, device="cuda")
    w = {(n, k): torch.randn(n, k, device="cuda", generator=g) / k ** 0.5 for n, k in ((512, 256), (512, 512), (256, 512))}
    bias = torch.randn(512, device="cuda", generator=g) * 0.1
    ws = torch.empty(3 * 512 * 512, device="cuda", dtype=torch.int16)
    part = torch.empty(256 * 512 * 512, device="cuda")
    cases = []
    for (n, k) in ((512, 256), (512, 512), (256, 512)):
        x = c256 if k == 256 else a512
        cases.append((f"FWD {k}->{n}", 2.0 * rows * k * n,
                      lambda lib, old, x=x, n=n, k=k: lib.vss_linear_tanh_bf16x6(
                          st, rows, k, n, x.data_ptr(), w[(n, k)].data_ptr(), bias.data_ptr(), out.data_ptr(),
                          *([] if old else [ws.data_ptr()]))))
    for (kn, n) in ((256, 512), (512, 512), (512, 256)):
        # backward from a layer of width kn (weight (kn, n)) into a tanh layer of width n
        gz = b512[:, :kn] if kn == 512 else c256
        y = a512 if n == 512 else c256
        wt = w[(kn, n)].t().contiguous()
        cases.append((f"BWD {kn}->{n}", 2.0 * rows * kn * n,
                      lambda lib, old, gz=gz.contiguous(), y=y, wt=wt, kn=kn, n=n: lib.vss_linear_tanh_backward_bf16x6(
                          st, rows, kn, n, gz.data_ptr(), wt.data_ptr(), y.data_ptr(), out.data_ptr(), part.data_ptr(),
                          *([] if old else [ws.data_ptr()]))))
    for (n, k) in ((512, 256), (512, 512), (256, 512)):
        gg = b512 if n == 512 else c256
        x = c256 if k == 256 else a512
        cases.append((f"WGRAD {n}x{k}", 2.0 * rows * k * n,
                      lambda lib, old, gg=gg, x=x, n=n, k=k: lib.vss_weight_grad_bf16x6(
                          st, rows, n, k, gg.data_ptr(), x.data_ptr(), part.data_ptr())))
    # every variant's results bitwise against the product library's (same arithmetic, same order)
    for name, _, fn in cases:
        out.zero_()
        part.zero_()
        fn(L[0][1], L[0][2])
        torch.cuda.synchronize()
        ref = (out.clone(), part.clone())
        for v, lib, old in L[1:]:
            out.zero_()
            part.zero_()
            fn(lib, old)
            torch.cuda.synchronize()
            o, q = torch.equal(out, ref[0]), torch.equal(part, ref[1])
            print(f"check {name:14s} {v}: output {'bit-exact' if o else 'DIFFERS'}, partials "
                  f"{'bit-exact' if q else 'differ (layout or order)'}", flush=True)
    # clocks up before the first measured case (the first case otherwise measures the ramp)
    for _ in range(3):
        for _, fn in [(c[0], c[2]) for c in cases]:
            fn(L[0][1], L[0][2])
    torch.cuda.synchronize()
    for name, fl, fn in cases:
        res = {v: [] for v, _, _ in L}
        for _ in range(rounds):
            for v, lib, old in L:
                res[v].append(timeit(lambda: fn(lib, old), 5))
        line = "  ".join(f"{v} {statistics.median(t):6.0f} us {fl / statistics.median(t) / 1e6:5.1f} TF" for v, t in res.items())
        print(f"{name:14s} {line}", flush=True)


if __name__ == "__main__":
    main()
