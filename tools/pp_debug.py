#!/usr/bin/env python3
"""Debug-only: where the pp backward differs from fp64 (rows / features with NaN or large error), with a
sentinel-filled output (rows never written keep 12345.0)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import linear_tanh_backward_x6  # noqa: E402

for rows, k_next, n in [(256, 128, 256), (256, 128, 256), (384, 128, 256), (640, 128, 256), (256, 192, 256),
                        (512, 128, 256), (256, 64, 256)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    gz = torch.randn(rows, k_next, device="cuda", generator=g) * 1e-3
    w = torch.randn(k_next, n, device="cuda", generator=g) / k_next ** 0.5
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    ref = (gz.double() @ w.double()) * (1 - y.double() ** 2)
    out = torch.full((rows, n), 12345.0, device="cuda")
    _, db = linear_tanh_backward_x6(gz, w, y, out=out)
    torch.cuda.synchronize()
    sent = out == 12345.0
    bad = ~torch.isfinite(out)
    err = (out.double() - ref).abs() / ref.abs().max()
    big = (err > 1e-5) & ~sent
    print(f"rows {rows} k_next {k_next} n {n}: unwritten {int(sent.sum())}, nonfinite {int(bad.sum())}, "
          f"wrong {int(big.sum())}", flush=True)
    for name, m in (("unwritten", sent), ("wrong", big)):
        if m.any():
            r = m.any(1).nonzero().squeeze(1)
            c = m.any(0).nonzero().squeeze(1)
            print(f"  {name} rows {r[:4].tolist()}..{r[-1:].tolist()} ({r.numel()}) cols {c[:4].tolist()}..({c.numel()})",
                  flush=True)
