#!/usr/bin/env python3
"""Profiling-only: where the PPO loop's device memory sits after its first update (ENV_ID sa / dma, NUM_ENVS):
the caching allocator's segments summed by memory pool (the default pool vs the minibatch graph's MemPool) and
by stream, with the allocated bytes inside them, plus the allocator's peak counters."""
import collections
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
from vss_amd.minibatch import disable_graph_packet_capture  # noqa: E402

disable_graph_packet_capture()
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402

env_id = os.environ.get("ENV_ID", "dma")
num_envs = int(os.environ.get("NUM_ENVS", 3 * 65536 if env_id == "dma" else 65536))
args = P.parse_args(["--env-id", env_id, "--num-envs", str(num_envs), "--num-updates", "1", "--log", "false",
                     "--seed", "1"])
out = {}


def summary(tag):
    by_pool = collections.defaultdict(lambda: [0, 0, 0])
    for seg in torch.cuda.memory_snapshot():
        key = str(seg.get("segment_pool_id", "?"))
        by_pool[key][0] += seg["total_size"]
        by_pool[key][1] += seg["allocated_size"]
        by_pool[key][2] += 1
    st = torch.cuda.memory_stats()
    out[tag] = {"pools_gib": {k: {"reserved": v[0] / 2 ** 30, "allocated": v[1] / 2 ** 30, "segments": v[2]}
                              for k, v in by_pool.items()},
                "reserved_gib": st["reserved_bytes.all.current"] / 2 ** 30,
                "allocated_gib": st["allocated_bytes.all.current"] / 2 ** 30,
                "peak_reserved_gib": st["reserved_bytes.all.peak"] / 2 ** 30,
                "peak_allocated_gib": st["allocated_bytes.all.peak"] / 2 ** 30,
                "num_alloc_retries": st.get("num_alloc_retries", 0), "num_ooms": st.get("num_ooms", 0)}
    print(tag, json.dumps(out[tag]), flush=True)


def on_update(rec, agent):
    summary("after_update_1")
    return False


P.train(args, on_update=on_update)
summary("after_train")
