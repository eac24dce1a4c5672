#!/usr/bin/env python3
"""Profiling-only: vss_sum_parts on the update's job shapes at 65,536 envs (one MLP backward): each job
alone and all together, HIP events over REPS launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import sum_parts  # noqa: E402

reps = int(os.environ.get("REPS", 20))
dev = "cuda"
shapes = {"wgrad 256x512 (64 parts)": (64, 256, 512), "wgrad 512x512 (32 parts)": (32, 512, 512),
          "wgrad 512x256 (64 parts)": (64, 512, 256), "first layer 256x52 (256 parts)": (256, 256, 52),
          "bias 512 (128 parts)": (128, 512), "bias 256 (256 parts)": (256, 256), "out dW 2x256 (64 parts)": (64, 2, 256)}
jobs = {k: (torch.randn(*s, device=dev), torch.empty(*s[1:], device=dev)) for k, s in shapes.items()}


def timed(js):
    sum_parts(js)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        sum_parts(js)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for k, j in jobs.items():
    nbytes = j[0].numel() * 4
    us = timed([j])
    print(f"{k}: {us:.1f} us ({nbytes / us / 1e3:.2f} TB/s)", flush=True)
allj = list(jobs.values())
us = timed(allj)
print(f"all {len(allj)} jobs in one launch: {us:.1f} us ({sum(j[0].numel() * 4 for j in allj) / us / 1e3:.2f} TB/s)")
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record()
for _ in range(reps):
    for p, o in allj:
        torch.sum(p, 0, out=o)
t1.record()
torch.cuda.synchronize()
print(f"torch.sum one per job: {t0.elapsed_time(t1) / reps * 1e3:.1f} us")
