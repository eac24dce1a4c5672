#!/usr/bin/env python3
"""Profiling-only: per-update rollout / update times of the PPO loop (ENV_ID sa|cma|dma, NUM_ENVS rows, default SA at 65,536), run
standalone (PROBE_ENV=0) or after creating a 65,536-field FULL env and stepping it the way
bench.py does first (PROBE_ENV=1)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402

PACKET_CAPTURE_OFF = P.disable_graph_packet_capture()  # an entry point: before anything initialises the GPU

if os.environ.get("PROBE_ENV", "0") == "1":
    from envs.vss import VSS, default_cfg
    env = VSS(default_cfg(65536), "cuda:0", "cuda:0", 0, True, False, False)
    a = torch.rand(65536, 2, 3, 2, device="cuda") * 2 - 1
    for _ in range(300):
        env.step(a)
    torch.cuda.synchronize()
if os.environ.get("PROBE_RANDPERM") == "arange":  # upper bound of a free permutation: no shuffle at all
    torch.randperm = lambda n, device=None, generator=None, **kw: torch.arange(n, device=device)  # noqa: E731
args = P.parse_args(["--env-id", os.environ.get("ENV_ID", "sa"), "--num-envs", os.environ.get("NUM_ENVS", "65536"), "--num-updates", os.environ.get("UPDATES", "3"),
                     "--log", os.environ.get("PROBE_LOG", "false"), "--seed", "1", "--save-path", "/tmp/runs"])
_, hist = P.train(args)
for h in hist:
    if "update_s" in h:
        print(f"PROBE_ENV={os.environ.get('PROBE_ENV', '0')} packet_capture_off={PACKET_CAPTURE_OFF} log={args.log} update {h['update']} rollout {h['rollout_s']:.3f} "
              f"update {h['update_s']:.3f}", flush=True)
