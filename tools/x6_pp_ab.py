#!/usr/bin/env python3
"""Profiling-only: the update's forward / backward / weight-gradient x6 shapes at ROWS rows (default
2,097,152), timed with HIP events over REPS launches each, in the kernel variant the environment selects
(round 5: VSS_X6_PRIO=1 raises the second half of each block's waves to s_setprio 1).  Prints
fp32-equivalent TF per shape and a checksum of each output (compare runs for the same bits)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import linear_tanh_backward_x6, linear_tanh_out_x6, linear_tanh_x6, weight_grad_x6  # noqa: E402

rows = int(os.environ.get("ROWS", 2097152))
reps = int(os.environ.get("REPS", 10))
tag = f"PRIO={os.environ.get('VSS_X6_PRIO', '0')}"
g = torch.Generator(device="cuda").manual_seed(0)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def csum(t):
    return float(t.double().sum()), float(t.double().abs().sum())


for k, n in ((256, 512), (512, 512), (512, 256)):
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    y = torch.empty(rows, n, device="cuda")
    ms = timed(lambda: linear_tanh_x6(x, w, b, out=y))
    print(f"{tag} forward {k}->{n}: {ms:.3f} ms {2 * rows * k * n / ms / 1e9:.1f} TF  sum {csum(y)}", flush=True)
    if n == 256:
        wo = torch.randn(2, 256, device="cuda", generator=g) / 16
        bo = torch.zeros(2, device="cuda")
        res = {}
        ms = timed(lambda: res.update(o=linear_tanh_out_x6(x, w, b, wo, bo, out=y)))
        print(f"{tag} forward+out {k}->{n}: {ms:.3f} ms {2 * rows * k * n / ms / 1e9:.1f} TF  sum {csum(res['o'][1])}",
              flush=True)
    del x, y
    gn = torch.randn(rows, n, device="cuda", generator=g) * 1e-3
    wn = torch.randn(n, k, device="cuda", generator=g) / n ** 0.5
    yk = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    gz = torch.empty(rows, k, device="cuda")
    res = {}
    ms = timed(lambda: res.update(o=linear_tanh_backward_x6(gn, wn, yk, out=gz)))
    print(f"{tag} backward {k}<-{n}: {ms:.3f} ms {2 * rows * k * n / ms / 1e9:.1f} TF  sum {csum(gz)} db {csum(res['o'][1])}",
          flush=True)
    res = {}
    ms = timed(lambda: res.update(o=weight_grad_x6(gn, yk)))
    print(f"{tag} wgrad {n}x{k}: {ms:.3f} ms {2 * rows * k * n / ms / 1e9:.1f} TF  sum {csum(res['o'])}", flush=True)
    del gn, yk, gz
    torch.cuda.empty_cache()
