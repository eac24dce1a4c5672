#!/usr/bin/env python3
"""Profiling-only: the Agent's first layer forward, y = tanh(x W^T + b) (52 -> 256), on the fp32 MFMA
(vss_linear_tanh -> first_layer_kernel) and on the bf16 matrix cores (vss_first_layer_bf16x6), timed with
HIP events over REPS launches at the rollout's and the update's row counts; prints us per launch, the
algorithmic HBM rate ((52 + 256) x 4 B per row) and each one's max error against fp64."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import first_layer_x6, linear_tanh  # noqa: E402

reps = int(os.environ.get("REPS", 20))
tag = f"CFG={os.environ.get('VSS_FL_CFG', '1')}"
g = torch.Generator(device="cuda").manual_seed(0)
w = torch.randn(256, 52, device="cuda", generator=g) * (2 / 52) ** 0.5
b = torch.randn(256, device="cuda", generator=g) * 0.1


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for rows in (65536, 131072, 2097152):
    x = torch.randn(rows, 52, device="cuda", generator=g)
    y32, yx = torch.empty(rows, 256, device="cuda"), torch.empty(rows, 256, device="cuda")
    t32 = timed(lambda: linear_tanh(x, w, b, out=y32))
    tx6 = timed(lambda: first_layer_x6(x, w, b, out=yx))
    ref = torch.tanh(x[:65536].double() @ w.double().t() + b.double())
    e32 = float((y32[:65536].double() - ref).abs().max())
    ex6 = float((yx[:65536].double() - ref).abs().max())
    gbs = rows * (52 + 256) * 4 / 1e9
    print(f"{tag} rows {rows}: fp32 {t32:.1f} us ({gbs / t32 * 1e3:.2f} TB/s)  x6 {tx6:.1f} us "
          f"({gbs / tx6 * 1e3:.2f} TB/s)  max err fp32 {e32:.2e} x6 {ex6:.2e}", flush=True)
