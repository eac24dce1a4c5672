#!/usr/bin/env python3
"""Profiling-only: the PPO update's fused-epilogue GEMMs against what torch issues, at the update's
shapes (ROWS = 2,097,152 minibatch rows; the Agent's 52->256, 256->512, 512->512, 512->256 layers):

  forward   vss_linear_tanh           vs hipBLASLt addmm + torch tanh
  backward  vss_linear_tanh_backward  vs hipBLASLt mm (dX) + vss_tanh_grad_bias

Prints time, TFLOP/s of the GEMM part and the max deviation from torch.  `build name="-D..."`
builds knob variants of csrc/vss_update.hip into tools/_build/liblt_<name>.so, timed beside the
product library."""
import ctypes
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import _native as N  # noqa: E402
from vss_amd.update import tanh_grad_bias  # noqa: E402


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


def variants():
    out = [("product", N.load())]
    for path in sorted(glob.glob(os.path.join(REPO, "tools", "_build", "liblt_*.so"))):
        L = ctypes.CDLL(path)
        L.vss_linear_tanh.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 4
        L.vss_linear_tanh_backward_chunks.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
        L.vss_linear_tanh_backward_chunks.restype = ctypes.c_int64
        L.vss_linear_tanh_backward.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + \
            [ctypes.c_void_p] * 5
        out.append((os.path.basename(path)[6:-3], L))
    return out


def build(flags_by_name):
    src = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_update.hip")
    os.makedirs(os.path.join(REPO, "tools", "_build"), exist_ok=True)
    for name, flags in flags_by_name.items():
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", *flags,
                        "-o", os.path.join(REPO, "tools", "_build", f"liblt_{name}.so"), src], check=True)


def _bwd(libs, rows, st, g, kn, nn_):
    """backward through a layer with kn outputs into the tanh of a layer with nn_ outputs"""
    gz_next = torch.randn(rows, kn, device="cuda", generator=g) * 1e-3
    w_next = torch.randn(kn, nn_, device="cuda", generator=g) / kn ** 0.5
    yl = torch.tanh(torch.randn(rows, nn_, device="cuda", generator=g))
    out = torch.empty(rows, nn_, device="cuda")
    t_ref = timeit(lambda: tanh_grad_bias(gz_next.mm(w_next), yl))
    t_gemm = timeit(lambda: gz_next.mm(w_next))
    fl = 2.0 * rows * kn * nn_
    gbytes = rows * (kn + 2 * nn_) * 4 / 1e9
    print(f"BWD K {kn:3d} N {nn_:3d}: torch mm + tanh_grad_bias {t_ref:7.0f} us (mm {t_gemm:7.0f} us = "
          f"{fl / t_gemm / 1e6:5.1f} TF)", flush=True)
    ref, ref_bias = tanh_grad_bias(gz_next.mm(w_next), yl)
    w_t = w_next.t().contiguous()
    for name, lib in libs:
        part = torch.empty(lib.vss_linear_tanh_backward_chunks(rows, kn, nn_), nn_, device="cuda")
        out.zero_()
        t_ours = timeit(lambda: lib.vss_linear_tanh_backward(st, rows, kn, nn_, gz_next.data_ptr(), w_t.data_ptr(),
                                                             yl.data_ptr(), out.data_ptr(), part.data_ptr()))
        err = float((out - ref).abs().max())
        berr = float((part.sum(0) - ref_bias).abs().max() / ref_bias.abs().max())
        print(f"    {name:12s} {t_ours:7.0f} us = {fl / t_ours / 1e6:5.1f} TF  {gbytes / t_ours * 1e3:5.2f} TB/s   "
              f"max|diff| {err:.2e}   bias rel {berr:.1e}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return build({kv.split("=", 1)[0]: kv.split("=", 1)[1].split() for kv in sys.argv[2:]})
    libs = variants()
    rows = int(os.environ.get("ROWS", 2097152))
    st = torch.cuda.current_stream().cuda_stream
    print(f"rows {rows}", flush=True)
    for k, n in ((4, 256), (8, 256), (52, 256), (256, 512), (512, 512), (512, 256)):
        g = torch.Generator(device="cuda").manual_seed(k * n)
        x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
        w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
        b = torch.randn(n, device="cuda", generator=g) * 0.1
        y = torch.empty(rows, n, device="cuda")
        if k in (4, 8):  # the output layer's (zero-padded) backward only: gz_next (rows, k), y (rows, n)
            del x, y
            _bwd(libs, rows, st, g, k, n)
            continue
        t_ref = timeit(lambda: torch.addmm(b, x, w.t()).tanh_())
        t_gemm = timeit(lambda: torch.addmm(b, x, w.t()))
        fl = 2.0 * rows * k * n
        print(f"FWD K {k:3d} N {n:3d}: torch addmm+tanh {t_ref:7.0f} us (addmm {t_gemm:7.0f} us = {fl / t_gemm / 1e6:5.1f} TF)",
              flush=True)
        ref = torch.addmm(b, x, w.t()).tanh_()
        for name, lib in libs:
            y.zero_()
            t_ours = timeit(lambda: lib.vss_linear_tanh(st, rows, k, n, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                                        y.data_ptr()))
            err = float((y - ref).abs().max())
            print(f"    {name:12s} {t_ours:7.0f} us = {fl / t_ours / 1e6:5.1f} TF   max|diff| {err:.2e}", flush=True)
        del x, y, ref
        if k == 52:
            continue
        # backward through layer (n -> k) and the tanh of the layer below it: (rows, k) x (k, n)
        _bwd(libs, rows, st, g, n, k)


if __name__ == "__main__":
    main()
