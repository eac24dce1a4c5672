"""K = 16 rollout timed with its output buffers at different relative placements (profiling tool):
obs and terminal_obs carved out of one allocation, the second starting `skew` bytes past the end of
the first; each placement re-allocated REPS times (fresh physical pages)."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from envs.vss import VSS, default_cfg  # noqa: E402

N = int(os.environ.get("RS_FIELDS", 65536))
K = int(os.environ.get("RS_K", 16))
REPS = int(os.environ.get("RS_REPS", 3))
SKEWS = [int(s) for s in os.environ.get("RS_SKEWS", "-1,0,4096,65536,1048576,2097152,3145728").split(",")]


def main():
    dev = torch.device("cuda:0")
    cfg = default_cfg(N)
    cfg["env"]["seed"] = 5
    env = VSS(cfg, str(dev), str(dev), 0, True, False, False)
    gen = torch.Generator(device=dev).manual_seed(3)
    env.progress_buf.random_(0, int(env.max_episode_length), generator=gen)
    acts = torch.rand((K, N, 2, 3, 2), device=dev, generator=gen) * 2 - 1
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    obs_floats = K * N * 312
    for rep in range(REPS):
        for skew in SKEWS:
            if skew < 0:
                out = env.rollout(acts)  # the host layer's own allocation
            else:
                big = torch.empty(2 * obs_floats + skew // 4 + 64, device=dev)
                out = env.rollout(acts)
                out["obs"] = big[:obs_floats].view(K, N, 2, 3, 52)
                out["terminal_observation"] = big[obs_floats + skew // 4: 2 * obs_floats + skew // 4].view(K, N, 2, 3, 52)
            env.rollout(acts, out)
            torch.cuda.synchronize()
            launches = 12
            e0.record()
            for _ in range(launches):
                env.rollout(acts, out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / (launches * K) * 1e3
            res.append({"skew": skew, "rep": rep, "us_per_step": round(us, 2),
                        "obs_ptr_mod_2M": out["obs"].data_ptr() % (2 << 20),
                        "term_minus_obs": out["terminal_observation"].data_ptr() - out["obs"].data_ptr()})
            print(res[-1], flush=True)
            del out
            if skew >= 0:
                del big
            torch.cuda.empty_cache()
    print(json.dumps({"fields": N, "K": K, "results": res}), flush=True)


if __name__ == "__main__":
    main()
