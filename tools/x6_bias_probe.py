#!/usr/bin/env python3
"""Profiling-only: is the x6 GEMMs' rounding error biased?  tests/test_update_parity.py found the update's bias
gradients (column sums of the x6 backward outputs over 2,097,152 rows) 20-60 x further from fp64 than torch's
fp32 ones, while the weight gradients are within 1.6 x.  A column sum over n rows grows a BIASED per-element
error like n but an unbiased one like sqrt(n), so this measures, per GEMM path (x6, the fp32-MFMA kernel, torch
fp32 = hipBLASLt) on random data:

  bias   = mean(e * sign(ref)) / mean(|e|)   with e = out - ref64 (-1: always toward zero, 0: unbiased)
  colsum = relative error of the column sums over ROWS rows
  elem   = relative Frobenius error of the elements"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import update as U  # noqa: E402


def stats(out, ref):
    e = out.double() - ref
    return {"bias": float((e * torch.sign(ref)).mean() / e.abs().mean()),
            "offset": float(e.mean() / e.pow(2).mean().sqrt()),
            "colsum_offset": float(((out.double().sum(0) - ref.sum(0)) / ref.abs().sum(0)).mean()),
            "colsum": float((out.double().sum(0) - ref.sum(0)).norm() / ref.sum(0).norm()),
            "elem": float(e.norm() / ref.norm())}


def main():
    rows = int(os.environ.get("ROWS", "524288"))
    g = torch.Generator(device="cuda").manual_seed(3)
    res = {"rows": rows}
    # backward 512 <- 256: gz = (gn W) (1 - y^2), gn (rows, 256), W (256, 512)
    gn = torch.randn(rows, 256, device="cuda", generator=g) * 1e-3
    w = torch.randn(256, 512, device="cuda", generator=g) / 16
    y = torch.tanh(torch.randn(rows, 512, device="cuda", generator=g))
    ref = (gn.double() @ w.double()) * (1 - y.double() ** 2)
    res["backward_x6"] = stats(U.linear_tanh_backward_x6(gn, w, y)[0], ref)
    res["backward_fp32mfma"] = stats(U.linear_tanh_backward(gn, w, y)[0], ref)
    res["backward_torch"] = stats((gn @ w) * (1 - y * y), ref)
    # the bare product (no tanh derivative): the same GEMM with y = 0
    z = torch.zeros_like(y)
    ref0 = gn.double() @ w.double()
    res["product_x6"] = stats(U.linear_tanh_backward_x6(gn, w, z)[0], ref0)
    res["product_torch"] = stats(gn @ w, ref0)
    # bf16-exact operands: the split's mid / lo planes are zero, so any column-correlated error is the bf16
    # MFMA's own accumulation (hi x hi products are exact in fp32)
    gb, wb = gn.bfloat16().float(), w.bfloat16().float()
    refb = gb.double() @ wb.double()
    res["product_x6_bf16_exact_inputs"] = stats(U.linear_tanh_backward_x6(gb, wb, z)[0], refb)
    res["product_torch_bf16_exact_inputs"] = stats(gb @ wb, refb)
    # one K tile (K = 32: one MFMA per product and output) and K = 64
    for k in (64, 128):
        g1, w1 = gn[:, :k].contiguous(), w[:k].contiguous()
        r1 = g1.double() @ w1.double()
        res[f"product_x6_k{k}"] = stats(U.linear_tanh_backward_x6(g1, w1, z)[0], r1)
        res[f"product_torch_k{k}"] = stats(g1 @ w1, r1)
    # forward 512 -> 512: y = tanh(x W^T + b)
    x = torch.tanh(torch.randn(rows, 512, device="cuda", generator=g))
    w2 = torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(512, device="cuda", generator=g) * 0.1
    ref2 = torch.tanh(x.double() @ w2.double().t() + b.double())
    res["forward_x6"] = stats(U.linear_tanh_x6(x, w2, b), ref2)
    res["forward_torch"] = stats(torch.addmm(b, x, w2.t()).tanh_(), ref2)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
