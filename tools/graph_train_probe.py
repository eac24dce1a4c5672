#!/usr/bin/env python3
"""Debug-only: train() with every MinibatchGraph replay checked against the eager minibatch step
on the same static inputs (gradients and losses), printing the first minibatches' differences."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from vss_amd import minibatch as MBM, mlp as MLP  # noqa: E402

_orig = MBM.MinibatchGraph.run
_count = [0]


def run(self, *a):
    st = _orig(self, *a)
    g_flat, g_st = self.flat.flat.clone(), [t.clone() for t in st]
    e_st = self._body()
    e_flat = self.flat.flat.clone()
    n = _count[0]
    _count[0] += 1
    if n < 12 or n % 8 == 0:
        print(f"minibatch {n}: max |grad diff| {(g_flat - e_flat).abs().max().item():.3e} "
              f"|grad| {e_flat.abs().max().item():.3e}  graph losses {[round(float(t), 5) for t in g_st]}  "
              f"eager {[round(float(t), 5) for t in e_st]}", flush=True)
    self.flat.flat.copy_(g_flat)
    return st


MBM.MinibatchGraph.run = run
args = P.parse_args(["--env-id", "sa", "--num-envs", os.environ.get("NUM_ENVS", "65536"), "--num-updates",
                     os.environ.get("UPDATES", "1"), "--log", "false", "--seed", "1", "--save-path", "/tmp/runs"])
_, hist = P.train(args)
for h in hist:
    print({k: h[k] for k in ("update", "approx_kl", "clipfrac", "v_loss", "update_s")}, flush=True)
