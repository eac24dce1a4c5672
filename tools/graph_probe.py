#!/usr/bin/env python3
"""Debug-only: the PPO update through MinibatchGraph vs eager on synthetic batches of several
minibatch sizes (one epoch, 2 minibatches): max parameter difference and the first-minibatch
losses of each, to locate a size where the captured step departs from the eager one."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from vss_amd import minibatch as MBM, mlp as MLP  # noqa: E402
from envs._gym import Box  # noqa: E402


def agent():
    from collections import namedtuple
    import numpy as np
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    torch.manual_seed(42)
    return P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (2,)))).cuda()


def main():
    if os.environ.get("SYNC_REPLAY"):  # wait for every replay before the eager work after it
        orig = MBM.MinibatchGraph.run

        def run(self, *a):
            st = orig(self, *a)
            torch.cuda.synchronize()
            return st
        MBM.MinibatchGraph.run = run
    if os.environ.get("NOSPLITK"):
        MLP.SPLITK_MIN_ROWS = 1 << 62  # the first layer's weight gradient as one mm instead of bmm + sum
    for mb in [int(v) for v in os.environ.get("MBS", "16384,32768,65536,262144,2097152").split(",")]:
        n = int(os.environ.get("NMB", 2)) * mb
        args = P.parse_args([])
        args.update_epochs = int(os.environ.get("EPOCHS", 1))
        args.num_minibatches = int(os.environ.get("NMB", 2))
        g = torch.Generator(device="cuda").manual_seed(3)
        obs = torch.randn(n, 52, device="cuda", generator=g)
        act = torch.randn(n, 2, device="cuda", generator=g) * 0.5
        logp, adv, ret, val = (torch.randn(n, device="cuda", generator=g) for _ in range(4))
        logp -= 3.0
        out = []
        for use_graph in (False, True):
            a = agent()
            flat = P.FlatGrads(a)
            opt = torch.optim.Adam(a.parameters(), lr=1e-3, eps=1e-5)
            graph = P.make_minibatch_graph(a, flat, args, n, (52,), (2,), "cuda") if use_graph else None
            st = P.ppo_update(a, opt, flat, args, obs, logp, act, adv, ret, val,
                              gen=torch.Generator(device="cuda").manual_seed(7), graph=graph)
            out.append((torch.cat([p.detach().reshape(-1) for p in a.parameters()]), st, flat.flat.clone()))
            del graph
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        d = (out[0][0] - out[1][0]).abs().max().item()
        dg = (out[0][2] - out[1][2]).abs().max().item()
        s0 = {k: round(float(v), 6) for k, v in out[0][1].items()}
        s1 = {k: round(float(v), 6) for k, v in out[1][1].items()}
        print(f"mb {mb}: max |param diff| {d:.3e}  max |grad diff| {dg:.3e}\n  eager {s0}\n  graph {s1}", flush=True)


if __name__ == "__main__":
    main()
