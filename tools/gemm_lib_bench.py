#!/usr/bin/env python3
"""Profiling-only: the PPO update's forward / input-gradient GEMM shapes (2,097,152 rows) under
torch's two ROCm BLAS back-ends (hipBLASLt = "cublaslt", rocBLAS = "cublas")."""
import torch

M = 2_097_152


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    torch.manual_seed(0)
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        for fin, fout in ((256, 512), (512, 512), (512, 256)):
            x = torch.randn(M, fin, device="cuda")
            w = torch.randn(fout, fin, device="cuda")
            b = torch.randn(fout, device="cuda")
            gy = torch.randn(M, fout, device="cuda")
            tf = t(lambda: torch.addmm(b, x, w.t()))
            tb = t(lambda: gy.mm(w))
            fl = 2 * M * fin * fout / 1e12
            print(f"{lib:9s} {fin}x{fout}: forward {tf:.2f} ms ({fl / tf * 1e3:.0f} TF), dX {tb:.2f} ms ({fl / tb * 1e3:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
