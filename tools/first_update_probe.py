#!/usr/bin/env python3
"""Profiling-only: where the PPO loop's first update loses time against the steady state (round-4
VERDICT: wall_s_per_update[0] 3.27 s vs 2.44 s, profiles/r04_ppo_65536_first_updates_gaps.txt).

Runs the SA train loop (65,536 envs by default, NUM_UPDATES updates) and prints, per update, the train
clock, rollout and update times and the caching allocator's device-malloc count (segments created) and
bytes reserved, so the first-use cost splits into allocation and the rest.  Knobs (environment):
  PRE_RESERVE_GB  allocate and free this many GB through torch's caching allocator before train()
  NUM_ENVS, NUM_UPDATES
Run it under `rocprofv3 --hip-trace --kernel-trace` to see which HIP API calls take the time."""
import os
import sys
import time

T_START = time.perf_counter()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402

PACKET_CAPTURE_OFF = P.disable_graph_packet_capture()


def mem():
    st = torch.cuda.memory_stats()
    return int(st.get("segment.all.allocated", 0)), torch.cuda.memory_reserved() / 1e9


def main():
    n = int(os.environ.get("NUM_ENVS", "65536"))
    upd = int(os.environ.get("NUM_UPDATES", "3"))
    torch.cuda.init()
    t_init = time.perf_counter() - T_START
    gb = float(os.environ.get("PRE_RESERVE_GB", "0"))
    t0 = time.perf_counter()
    if gb > 0:
        x = torch.empty(int(gb * 1e9) // 4, dtype=torch.float32, device="cuda")
        del x
        torch.cuda.synchronize()
    t_res = time.perf_counter() - t0
    print(f"packet_capture_off={PACKET_CAPTURE_OFF} process->cuda init {t_init:.2f} s, pre-reserve {gb} GB "
          f"{t_res:.2f} s, segments/reserved {mem()}", flush=True)
    args = P.parse_args(["--env-id", "sa", "--num-envs", str(n), "--num-updates", str(upd), "--log", "false",
                         "--seed", "1"])
    marks = []

    def on_update(rec, agent):
        marks.append((rec["update"], rec["wall_s"], rec["rollout_s"], rec["update_s"], *mem()))

    t0 = time.perf_counter()
    P.train(args, on_update=on_update)
    call = time.perf_counter() - t0
    prev = 0.0
    for u, wall, roll, up, seg, res in marks:
        print(f"update {u}: clock {wall:.3f} s (+{wall - prev:.3f}), rollout {roll:.3f}, update {up:.3f}, "
              f"segments {seg}, reserved {res:.1f} GB", flush=True)
        prev = wall
    print(f"train() call {call:.2f} s", flush=True)


if __name__ == "__main__":
    main()
