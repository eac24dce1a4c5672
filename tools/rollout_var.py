"""Does the episode-progress distribution move the step / rollout timings?  (profiling tool)

FULL single-step launches and K = 16 rollout launches at 65,536 fields, each timed with HIP events
over 12 launches (rollout) or 192 launches (step), from three starting states:
  fresh   -- every field at progress 0 (no time-out inside the window, goal resets only)
  desync  -- progress uniform over [0, maxEpisodeLength) (a running training loop: ~1/400 of the
             fields time out per step)
  burst   -- every field at maxEpisodeLength - 50 (all fields time out at the same step, inside
             the window)
Each state is re-created (state reset, progress set) before each of REPS repetitions."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from envs.vss import VSS, default_cfg  # noqa: E402

N = int(os.environ.get("RV_FIELDS", 65536))
K = 16
REPS = int(os.environ.get("RV_REPS", 3))


def set_state(env, how: str, gen):
    env.reset_buf.fill_(1)
    env.reset_dones()
    L = int(env.max_episode_length)
    if how == "fresh":
        env.progress_buf.zero_()
    elif how == "desync":
        env.progress_buf.random_(0, L, generator=gen)
    else:
        env.progress_buf.fill_(L - 50)
    env.reset_buf.zero_()
    torch.cuda.synchronize()


def main():
    dev = torch.device("cuda:0")
    cfg = default_cfg(N)
    cfg["env"]["seed"] = 5
    env = VSS(cfg, str(dev), str(dev), 0, True, False, False)
    gen = torch.Generator(device=dev).manual_seed(3)
    acts = torch.rand((K, N, 2, 3, 2), device=dev, generator=gen) * 2 - 1
    out = env.rollout(acts)
    pool = [torch.rand((N, 2, 3, 2), device=dev, generator=gen) * 2 - 1 for _ in range(16)]
    res = {}
    for how in ("fresh", "desync", "burst"):
        for rep in range(REPS):
            # rollout: 12 launches x 16 steps = 192 steps
            set_state(env, how, gen)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(12):
                env.rollout(acts, out)
            e1.record()
            torch.cuda.synchronize()
            r_us = e0.elapsed_time(e1) / (12 * K) * 1e3
            resets = int((out["dones"] != 0).sum()) if isinstance(out, dict) and "dones" in out else None
            # single steps: 192 launches
            set_state(env, how, gen)
            e0.record()
            for k in range(12 * K):
                env.step(pool[k % 16])
            e1.record()
            torch.cuda.synchronize()
            s_us = e0.elapsed_time(e1) / (12 * K) * 1e3
            res.setdefault(how, []).append({"rollout_us_per_step": round(r_us, 2), "step_us_incl_wrapper": round(s_us, 2),
                                            "last_launch_resets": resets})
            print(how, rep, res[how][-1], flush=True)
    print(json.dumps({"fields": N, "K": K, "results": res}), flush=True)


if __name__ == "__main__":
    main()
