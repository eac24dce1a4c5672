#!/usr/bin/env python3
"""Profiling-only: the product's x6 backward 512 <- 256 (vss_linear_tanh_backward_bf16x6 at 2,097,152 rows) timed
the way tools/x6_buildup.hip times its stages (1 s warm-up, then >= 2 s of back-to-back launches, HIP events), on
random data, so the build-up's last stage and the product kernel can be compared on one box."""
import os
import sys
import json

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import update as U  # noqa: E402

rows, k_next, n = 2097152, 256, 512
g = torch.Generator(device="cuda").manual_seed(1)
gn = torch.rand(rows, k_next, device="cuda", generator=g) * 2 - 1
w = (torch.rand(k_next, n, device="cuda", generator=g) * 2 - 1) / 16
y = torch.rand(rows, n, device="cuda", generator=g) * 2 - 1
out = torch.empty(rows, n, device="cuda")
planes = U.weight_planes([(w, True)])[0]


def launch():
    U.linear_tanh_backward_x6(gn, w, y, out=out, planes=planes, defer=[])




def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for seconds in (1.0, 2.0):
        launches, ms = 0, 0.0
        e0.record()
        while ms < seconds * 1e3:
            for _ in range(10):
                fn()
            launches += 10
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
    return launches, ms / launches


launches, per = timed(launch)
tf = 2.0 * rows * n * k_next / (per * 1e-3) / 1e12
print(json.dumps({"stage": "product vss_linear_tanh_backward_bf16x6 512<-256", "launches": launches, "ms_per_launch": per,
                  "x6_tflops": tf, "frac_of_x6_peak": tf / (2500.0 / 6),
                  "note": "wall includes the defer=[] partial-sum path (no reduction launch) per call"}), flush=True)
# the forward 512 -> 512 (the bench's update_gemm_roofline shape)
del gn, out
x = torch.tanh(torch.randn(rows, 512, device="cuda", generator=g))
w2 = torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5
b2 = torch.zeros(512, device="cuda")
y2 = torch.empty(rows, 512, device="cuda")
p2 = U.weight_planes([(w2, False)])[0]
launches, per = timed(lambda: U.linear_tanh_x6(x, w2, b2, out=y2, planes=p2))
tf = 2.0 * rows * 512 * 512 / (per * 1e-3) / 1e12
print(json.dumps({"stage": "product vss_linear_tanh_bf16x6 512->512", "launches": launches, "ms_per_launch": per,
                  "x6_tflops": tf, "frac_of_x6_peak": tf / (2500.0 / 6)}), flush=True)
# the fused loss launches (the last hidden layer 512 -> 256 with the output layer and the loss, EPI_LOSS_A /
# EPI_LOSS_C) beside the plain forward 512 -> 256 of the same shape: what the loss epilogue costs per launch
del y2
x3 = x
w3 = torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5
b3 = torch.zeros(256, device="cuda")
p3 = U.weight_planes([(w3, False)])[0]
y3 = torch.empty(rows, 256, device="cuda")
launches, per = timed(lambda: U.linear_tanh_x6(x3, w3, b3, out=y3, planes=p3))
tf = 2.0 * rows * 256 * 512 / (per * 1e-3) / 1e12
print(json.dumps({"stage": "product vss_linear_tanh_bf16x6 512->256", "launches": launches, "ms_per_launch": per,
                  "x6_tflops": tf, "frac_of_x6_peak": tf / (2500.0 / 6)}), flush=True)
del y3
real = rows - 32  # padding rows at the end, as a padded minibatch has
act = torch.randn(rows, 2, device="cuda", generator=g) * 0.3
logp, adv = torch.randn(rows, device="cuda", generator=g) - 1, torch.randn(rows, device="cuda", generator=g)
ret, val = torch.randn(rows, device="cuda", generator=g), torch.randn(rows, device="cuda", generator=g)
ls = torch.zeros(1, 2, device="cuda")
for actor, k_out in ((True, 2), (False, 1)):
    wo = torch.randn(k_out, 256, device="cuda", generator=g) / 16
    bo = torch.zeros(k_out, device="cuda")
    kw = dict(act=act, logp=logp, adv=adv, logstd=ls) if actor else dict(ret=ret, val=val, clip_vloss=True)
    launches, per = timed(lambda: U.linear_tanh_loss_x6(x3, w3, b3, wo, bo, real, actor, planes=p3, defer=[], **kw))
    tf = 2.0 * rows * 256 * 512 / (per * 1e-3) / 1e12
    print(json.dumps({"stage": f"product vss_linear_tanh_loss_bf16x6 512->256 {'actor' if actor else 'critic'}",
                      "launches": launches, "ms_per_launch": per, "x6_tflops": tf,
                      "frac_of_x6_peak": tf / (2500.0 / 6)}), flush=True)
