#!/usr/bin/env python3
"""Profiling-only: time variants of csrc/vss_update.hip (VSS_TG_* knobs) against torch's
tanh_backward + bias reduction at the PPO update's shapes (2,097,152 rows x 256 / 512 columns).

    python tools/tanh_grad_bench.py build    # here (hipcc), into tools/_build/libtg_<name>.so
    python tools/tanh_grad_bench.py          # on the GPU box
"""
import ctypes
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# measured (MI355X, 2,097,152 x 512): u8w4 2,385 us, u8w4nt 2,407, u4w8 2,418, u16w2 2,448,
# u8w4b4k 2,372, u8w4b1k 2,404; torch tanh_backward 2,155 (+ sum 2,935)
VARIANTS = {"u8w4": [], "u8w4nt": ["-DVSS_TG_NT=1"], "u4w8": ["-DVSS_TG_U=4", "-DVSS_TG_WAVES=8"],
            "u8w4b4k": ["-DVSS_TG_MAXBLK=4096"], "u16w2": ["-DVSS_TG_U=16", "-DVSS_TG_WAVES=2"],
            "u8w4b1k": ["-DVSS_TG_MAXBLK=1024"]}


def build():
    src = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_update.hip")
    os.makedirs(os.path.join(REPO, "tools", "_build"), exist_ok=True)
    for k, flags in VARIANTS.items():
        out = os.path.join(REPO, "tools", "_build", f"libtg_{k}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                        *flags, "-o", out, src], check=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return build()
    import torch
    rows = 2097152
    for cols in (512, 256):
        y = torch.tanh(torch.randn(rows, cols, device="cuda"))
        gy = torch.randn(rows, cols, device="cuda")
        gz = torch.empty_like(y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def timeit(fn, reps=10):
            fn()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps * 1e3

        t = timeit(lambda: torch.ops.aten.tanh_backward(gy, y).sum(0))
        tb = timeit(lambda: torch.ops.aten.tanh_backward(gy, y))
        nbytes = rows * cols * 12
        print(f"cols {cols}: torch tanh_backward {tb:.0f} us ({nbytes / tb / 1e6:.2f} TB/s), + sum {t:.0f} us")
        for path in sorted(glob.glob(os.path.join(REPO, "tools", "_build", "libtg_*.so"))):
            L = ctypes.CDLL(path)
            L.vss_tanh_grad_chunks.argtypes = [ctypes.c_int64, ctypes.c_int32]
            L.vss_tanh_grad_chunks.restype = ctypes.c_int64
            L.vss_tanh_grad_bias.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 4
            part = torch.empty((L.vss_tanh_grad_chunks(rows, cols), cols), device="cuda")
            st = torch.cuda.current_stream().cuda_stream
            fn = lambda: L.vss_tanh_grad_bias(st, rows, cols, gy.data_ptr(), y.data_ptr(), gz.data_ptr(),  # noqa: E731
                                              part.data_ptr())
            tk = timeit(fn)
            ok = torch.allclose(part.sum(0), torch.ops.aten.tanh_backward(gy, y).sum(0), rtol=1e-3, atol=1e-1)
            print(f"   {os.path.basename(path)[6:-3]:10s} {tk:7.0f} us ({nbytes / tk / 1e6:.2f} TB/s) ok={ok}")


if __name__ == "__main__":
    main()
