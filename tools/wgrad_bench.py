#!/usr/bin/env python3
"""Profiling-only: time the PPO update's weight-gradient GEMMs dW = dY^T X (K = 2,097,152
minibatch rows) as autograd issues them vs split-K forms (bmm over row chunks + sum)."""
import json
import torch

M = 2_097_152
SHAPES = [(52, 256), (256, 512), (512, 512), (512, 256), (256, 2), (256, 1)]


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
    res = {}
    for fin, fout in SHAPES:
        x = torch.randn(M, fin, device="cuda")
        dy = torch.randn(M, fout, device="cuda")
        r = {"mm_dyT_x": t(lambda: dy.t().mm(x)), "mm_xT_dy_T": t(lambda: x.t().mm(dy).t())}
        for s in (8, 16, 32, 64, 128):
            r[f"bmm_split{s}"] = t(lambda s=s: torch.bmm(dy.view(s, M // s, fout).transpose(1, 2), x.view(s, M // s, fin)).sum(0))
        ref = dy.t().mm(x)
        r["max_rel_err_split32"] = float(((torch.bmm(dy.view(32, M // 32, fout).transpose(1, 2), x.view(32, M // 32, fin)).sum(0) - ref).abs().max() / ref.abs().max()))
        r["gflop"] = 2 * M * fin * fout / 1e9
        res[f"{fin}x{fout}"] = r
        print(f"{fin}x{fout}", {k: round(v, 3) for k, v in r.items()}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
