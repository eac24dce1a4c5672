#!/usr/bin/env python3
"""Wall-clock to a trained policy: PPO at the reference's defaults
(ppo_continuous_action_isaacgym.py:51-117; only --num-envs and --env-id chosen here) until the
policy's evaluation score against the zero team (play.py / ppo…:380-461: goal-only rewards, the
trained policy as the blue team) reaches --target, checked every --eval-every updates on
--eval-matches matches of a separate evaluation env.  The training clock excludes the evaluations.
At the crossing the score is confirmed with the reference's 10,000 matches against the zero and the
OU teams.  One JSON line:

    python tools/time_to_score.py --env-id sa --num-envs 4095 [--target 0.9] [--max-steps 3e8]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))

import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from envs.vss import VSS, default_cfg  # noqa: E402
from envs.wrappers import random_ou  # noqa: E402
from play import get_team, play_matches  # noqa: E402


class LiveTeam:
    """The training agent as the blue team without a checkpoint round trip: SA drives robot 0 and
    OU noise the others (play.py:51-54), CMA one 6-vector for the team, DMA one row per robot."""

    def __init__(self, agent, env_id):
        self.agent, self.env_id = agent, env_id

    @torch.no_grad()
    def __call__(self, act, obs):
        n = obs.shape[0]
        if self.env_id == "sa":
            act.copy_(random_ou(act))
            act[:, 0, :] = self.agent.get_action_and_value(obs[:, 0, :])[0]
        elif self.env_id == "cma":
            act.copy_(self.agent.get_action_and_value(obs[:, 0, :])[0].view(-1, 3, 2))
        else:
            act.copy_(self.agent.get_action_and_value(obs.reshape(n * 3, -1))[0].view(n, 3, 2))


def main():
    P.disable_graph_packet_capture()  # an entry point: before anything initialises the GPU
    ap = argparse.ArgumentParser()
    ap.add_argument("--env-id", default="sa", choices=["sa", "cma", "dma"])
    ap.add_argument("--num-envs", type=int, default=4095)
    ap.add_argument("--target", type=float, default=0.9)
    ap.add_argument("--eval-every", type=int, default=10)
    ap.add_argument("--eval-matches", type=int, default=2000)
    ap.add_argument("--confirm-matches", type=int, default=10000)
    ap.add_argument("--eval-fields", type=int, default=4096)
    ap.add_argument("--max-steps", type=float, default=3e8)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    # no kernel warm-up: this clock starts before train() and keeps every first use, as in rounds 3-4
    args = P.parse_args(["--env-id", a.env_id, "--num-envs", str(a.num_envs), "--seed", str(a.seed),
                         "--log", "false", "--kernel-warmup", "false"])
    args.num_updates = int(a.max_steps // args.batch_size)
    cfg = default_cfg(a.eval_fields)
    cfg["env"]["seed"] = 1000 + a.seed
    ev = VSS(cfg, "cuda:0", "cuda:0", 0, True, False, False)
    ev.w_goal, ev.w_grad, ev.w_move, ev.w_energy = 1.0, 0.0, 0.0, 0.0  # evaluation rewards (ppo…:389-392)
    zero, ou = get_team("zero"), get_team("ou")
    state = {"eval_s": 0.0, "t0": time.time(), "curve": [], "hit": None}

    def on_update(rec, agent):
        if rec["update"] % a.eval_every:
            return False
        t = time.time()
        score, length = play_matches(ev, LiveTeam(agent, a.env_id), zero, a.eval_matches)
        state["eval_s"] += time.time() - t
        train_s = time.time() - state["t0"] - state["eval_s"]
        state["curve"].append({"update": rec["update"], "env_steps": rec["global_step"], "train_s": train_s,
                               "score_zero": score, "length": length, "mean_return": rec["mean_return"]})
        print(json.dumps(state["curve"][-1]), flush=True)
        if score >= a.target:
            state["hit"] = state["curve"][-1]
            return True
        return False

    agent, hist = P.train(args, on_update=on_update)
    out = {"env_id": a.env_id, "num_envs": a.num_envs, "batch": args.batch_size, "target_score_vs_zero": a.target,
           "eval_every_updates": a.eval_every, "eval_matches": a.eval_matches, "reached": state["hit"] is not None,
           "curve": state["curve"]}
    if state["hit"]:
        h = state["hit"]
        out.update(wallclock_to_target_s=h["train_s"], env_steps_to_target=h["env_steps"], updates_to_target=h["update"])
        live = LiveTeam(agent, a.env_id)
        out["confirm"] = {"matches": a.confirm_matches,
                          "score_zero": play_matches(ev, live, zero, a.confirm_matches)[0],
                          "score_ou": play_matches(ev, live, ou, a.confirm_matches)[0]}
    print("TIME_TO_SCORE " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
