"""K sweep of the K-step rollout kernel (profiling tool): µs per env step and the fraction of the
8 TB/s spec on the kernel's algorithmic bytes, at 65,536 fields, episodes desynchronised, HIP
events over `launches` launches; K = 1 is also compared with the single-step FULL launch."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from envs.vss import VSS, default_cfg  # noqa: E402

N = int(os.environ.get("RK_FIELDS", 65536))
KS = [int(k) for k in os.environ.get("RK_KS", "1,2,4,8,16,32").split(",")]
STEPS = 192


def algo_bytes(n, K):
    return n * (K * (48 + 1248 + 1248 + 96 + 8 + 1 + 4) + 368 + 32 + 8 + 48)


def main():
    dev = torch.device("cuda:0")
    cfg = default_cfg(N)
    cfg["env"]["seed"] = 5
    env = VSS(cfg, str(dev), str(dev), 0, True, False, False)
    gen = torch.Generator(device=dev).manual_seed(3)
    env.progress_buf.random_(0, int(env.max_episode_length), generator=gen)
    res = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pool = [torch.rand((N, 2, 3, 2), device=dev, generator=gen) * 2 - 1 for _ in range(16)]
    for rep in range(2):
        for k in range(16):
            env.step(pool[k])
        torch.cuda.synchronize()
        e0.record()
        for k in range(STEPS):
            env.step(pool[k % 16])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / STEPS * 1e3
        res.append({"K": "step", "rep": rep, "us_per_step": round(us, 2), "frac": round(3101 * N / (us * 1e-6) / 8e12, 4)})
        print(res[-1], flush=True)
        for K in KS:
            acts = torch.rand((K, N, 2, 3, 2), device=dev, generator=gen) * 2 - 1
            out = env.rollout(acts)
            env.rollout(acts, out)
            launches = max(2, STEPS // K)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(launches):
                env.rollout(acts, out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / launches
            res.append({"K": K, "rep": rep, "us_per_step": round(ms * 1e3 / K, 2),
                        "frac": round(algo_bytes(N, K) / (ms * 1e-3) / 8e12, 4)})
            print(res[-1], flush=True)
            del out, acts
    print(json.dumps({"fields": N, "results": res}), flush=True)


if __name__ == "__main__":
    main()
