#!/usr/bin/env python3
"""Profiling-only: vss_minibatch_gather at the SA update's shape (a 2,097,152-row minibatch of an 8,388,608-row
batch, 52 observation and 2 action floats per row) timed with HIP events over >= 2 s of launches, with the bytes it
moves (rows written once, rows read at 128-B line granularity, the indices)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.loss import minibatch_gather, minibatch_gather_parts  # noqa: E402

batch, mb, ow, aw = 8388608, 2097152, 52, 2
g = torch.Generator(device="cuda").manual_seed(0)
b_obs = torch.randn(batch, ow, device="cuda", generator=g)
b_act = torch.randn(batch, aw, device="cuda", generator=g)
b_s = [torch.randn(batch, device="cuda", generator=g) for _ in range(4)]
inds = torch.randperm(batch, device="cuda", generator=g)[:mb].contiguous()
obs, act = torch.empty(mb, ow, device="cuda"), torch.empty(mb, aw, device="cuda")
outs = [torch.empty(mb, device="cuda") for _ in range(4)]
part = torch.empty(minibatch_gather_parts(mb), 2, device="cuda", dtype=torch.float64)
fn = lambda: minibatch_gather(inds, b_obs, b_act, *b_s, obs, act, *outs, part)  # noqa: E731
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for seconds in (1.0, 2.0):
    n, ms = 0, 0.0
    e0.record()
    while ms < seconds * 1e3:
        for _ in range(20):
            fn()
        n += 20
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
per = ms / n
moved = mb * (4 * (ow + aw) + 4 * 4) * 2 + mb * 8
print(json.dumps({"kernel": "vss_minibatch_gather", "rows": mb, "batch": batch, "launches": n, "ms_per_launch": per,
                  "rows_bytes_read_plus_written_GBps": moved / per / 1e6}), flush=True)
