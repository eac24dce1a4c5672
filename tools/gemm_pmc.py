#!/usr/bin/env python3
"""Profiling-only: one fused-GEMM shape (GEMM_DIR=fwd|bwd, K, N env vars; 2,097,152 rows) launched
REPS times, for rocprofv3 --pmc / --kernel-trace runs of vss_linear_tanh / vss_linear_tanh_backward."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import linear_tanh, linear_tanh_backward  # noqa: E402

rows = int(os.environ.get("ROWS", 2097152))
k, n = int(os.environ.get("K", 512)), int(os.environ.get("N", 512))
reps = int(os.environ.get("REPS", 20))
g = torch.Generator(device="cuda").manual_seed(0)
if os.environ.get("GEMM_DIR", "fwd") == "fwd":
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.zeros(n, device="cuda")
    fn = lambda: linear_tanh(x, w, b)  # noqa: E731
else:
    gn = torch.randn(rows, k, device="cuda", generator=g)
    wn = torch.randn(k, n, device="cuda", generator=g) / k ** 0.5
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    fn = lambda: linear_tanh_backward(gn, wn, y)  # noqa: E731
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", rows, k, n, reps)
